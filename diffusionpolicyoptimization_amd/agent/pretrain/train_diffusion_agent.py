"""Pretraining agent (reference agent/pretrain/train_agent.py:61-187 and
train_diffusion_agent.py:16-120): epochs over a StitchedSequenceDataset, the diffusion loss
c_loss -> p_losses on the MI355X row-tile kernels (dppo_pretrain_minibatch), Keras-3 AdamW under
CosineDecayRestarts, an EMA copy of the network, Keras-3 .weights.h5 checkpoints per save_model_freq.

Differences from the reference, by design: t and noise come
from a seeded device generator instead of tf.random; wandb logging is not built (out of scope)."""
import logging
import os
import random

import numpy as np
import torch

from ...util.config import instantiate
from ...util.optim import AdamW
from ...util.scheduler import CosineDecayRestarts
from ...util.timer import Timer

log = logging.getLogger(__name__)


class EMA:
    """train_agent.py:46-59: ema = decay * ema + (1 - decay) * new."""

    def __init__(self, decay):
        self.decay = float(decay)

    def update_model_average(self, ema_params, params):
        ema_params.mul_(self.decay).add_(params, alpha=1.0 - self.decay)


class TrainDiffusionAgent:
    def __init__(self, cfg):
        self.cfg = cfg
        self.seed = int(cfg.get("seed", 42))
        random.seed(self.seed)
        np.random.seed(self.seed)
        torch.manual_seed(self.seed)
        self.model = instantiate(cfg.model)
        self.model._pretrain_init()
        self.ema = EMA(cfg.ema.decay)
        self.ema_params = self.model.params.clone()
        tr = cfg.train
        self.n_epochs = int(tr.n_epochs)
        self.batch_size = int(tr.batch_size)
        self.update_ema_freq = int(tr.update_ema_freq)
        self.epoch_start_ema = int(tr.epoch_start_ema)
        self.save_model_freq = int(tr.save_model_freq)
        self.log_freq = int(tr.get("log_freq", 1))
        self.logdir = cfg.logdir
        self.checkpoint_dir = os.path.join(self.logdir, "checkpoint")
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        self.dataset_train = instantiate(cfg.train_dataset)
        lr = float(tr.learning_rate)
        self.lr_scheduler = CosineDecayRestarts(lr, tr.lr_scheduler.first_cycle_steps, t_mul=1.0, m_mul=1.0,
                                                alpha=float(tr.lr_scheduler.min_lr) / lr)
        self.optimizer = AdamW(self.model.params, self.lr_scheduler, weight_decay=float(tr.weight_decay))
        self.epoch = 1

    def reset_parameters(self):
        self.ema_params.copy_(self.model.params)

    def step_ema(self):
        if self.epoch < self.epoch_start_ema:
            self.reset_parameters()
            return
        self.ema.update_model_average(self.ema_params, self.model.params)

    def save_model(self, epoch):
        ext = ".npz" if self.cfg.train.get("checkpoint_format", "h5") == "npz" else ".weights.h5"
        path = os.path.join(self.checkpoint_dir, f"state_{epoch}{ext}")   # agent/pretrain/train_agent.py:150-154
        self.model.save_network(path)
        saved = self.model.params.clone()
        self.model.params.copy_(self.ema_params)
        self.model.save_network(path.replace("state_", "ema_state_"))
        self.model.params.copy_(saved)
        log.info("Saved model to %s", path)

    def train_epoch(self):
        """One pass over the dataset: mean loss (train_diffusion_agent.py:57-76)."""
        m = self.model
        losses = []
        for batch in self.dataset_train.batches(self.batch_size):
            losses.append(m.c_loss(**batch))
            self.optimizer.apply_gradients(m.pre_grads)
            m.repack_network()
        return float(torch.stack(losses).mean()) if losses else float("nan")

    def run(self):
        timer = Timer()
        for _ in range(self.n_epochs):
            loss_train = self.train_epoch()
            if self.epoch % self.update_ema_freq == 0:
                self.step_ema()
            if self.epoch % self.save_model_freq == 0 or self.epoch == self.n_epochs:
                self.save_model(self.epoch)
            if self.epoch % self.log_freq == 0:
                log.info("%d: train loss %8.4f | t:%8.4f", self.epoch, loss_train, timer())
            self.epoch += 1
        return loss_train

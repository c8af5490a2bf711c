"""TrainPPOAgent (reference agent/finetune/train_ppo_agent.py:17-103): PPO hyper-parameters, the
single AdamW over [actor_ft | critic] with the cosine-warmup LR schedule, and the running reward
scaler (device-resident)."""
import logging

from ...util.optim import AdamW
from ...util.reward_scaling import RunningRewardScaler
from ...util.scheduler import CosineAnnealingWarmupRestarts2
from .train_agent import TrainAgent

log = logging.getLogger(__name__)


class TrainPPOAgent(TrainAgent):
    def __init__(self, cfg):
        super().__init__(cfg)
        self.logprob_batch_size = cfg.train.get("logprob_batch_size", 10000)
        if self.logprob_batch_size % self.n_envs_global:
            # the reference asserts here (train_ppo_agent.py:24-26); the fused log-prob pass has no
            # split, so the constraint is only reported
            log.warning("logprob_batch_size=%d not divisible by n_envs=%d (the reference would assert)",
                        self.logprob_batch_size, self.n_envs_global)
        self.gamma = cfg.train.gamma
        self.n_critic_warmup_itr = cfg.train.n_critic_warmup_itr
        self.actor_lr_scheduler = CosineAnnealingWarmupRestarts2(
            initial_learning_rate=cfg.train.actor_lr, first_cycle_steps=cfg.train.actor_lr_scheduler.first_cycle_steps,
            cycle_mult=1.0, max_lr=cfg.train.actor_lr, min_lr=cfg.train.actor_lr_scheduler.min_lr,
            warmup_steps=cfg.train.actor_lr_scheduler.warmup_steps, gamma=1.0)
        self.critic_lr_scheduler = CosineAnnealingWarmupRestarts2(
            initial_learning_rate=cfg.train.critic_lr, first_cycle_steps=cfg.train.critic_lr_scheduler.first_cycle_steps,
            cycle_mult=1.0, max_lr=cfg.train.critic_lr, min_lr=cfg.train.critic_lr_scheduler.min_lr,
            warmup_steps=cfg.train.critic_lr_scheduler.warmup_steps, gamma=1.0)
        # ONE Keras-3 AdamW for actor_ft AND critic at the actor LR; `decay=` is ignored by Keras 3 so
        # the default weight_decay 0.004 applies. Overridable for experiments.
        self.actor_optimizer = AdamW(self.model.train_params, learning_rate=self.actor_lr_scheduler,
                                     weight_decay=cfg.train.get("keras_weight_decay", 0.004),
                                     mode=cfg.train.get("optimizer_mode", "keras"))
        self.gae_lambda = cfg.train.get("gae_lambda", 0.95)
        self.target_kl = cfg.train.target_kl
        self.update_epochs = cfg.train.update_epochs
        self.ent_coef = cfg.train.get("ent_coef", 0)
        self.vf_coef = cfg.train.get("vf_coef", 0)
        self.model.vf_coef = self.vf_coef
        self.reward_scale_running = cfg.train.reward_scale_running
        if self.reward_scale_running:
            self.running_reward_scaler = RunningRewardScaler(self.n_envs, device=self.device)
        self.reward_scale_const = cfg.train.get("reward_scale_const", 1)
        self.use_bc_loss = cfg.train.get("use_bc_loss", False)
        self.bc_loss_coeff = cfg.train.get("bc_loss_coeff", 0)

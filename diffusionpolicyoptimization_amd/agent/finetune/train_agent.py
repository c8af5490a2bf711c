"""TrainAgent (reference agent/finetune/train_agent.py:15-167): seeding, env construction, model
instantiation, checkpoints — plus the MI355X data-parallel setup: one process per GPU, the env
batch sharded across ranks, torch.distributed over RCCL ("nccl") or gloo."""
import logging
import os
import random

import numpy as np
import torch
import torch.distributed as dist

from ...env.gym_utils import make_async
from ...util.config import instantiate
from ...util.dist import broadcast_, shard_envs

log = logging.getLogger(__name__)


def init_distributed():
    """(rank, world, local_rank, group) from the torchrun environment; world 1 when absent."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("DPPO_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, init_method="env://")
    return rank, world, local


class TrainAgent:
    def __init__(self, cfg):
        self.cfg = cfg
        self.rank, self.world_size, self.local_rank = init_distributed()
        dev = str(cfg.get("device", "cuda:0"))
        self.device = torch.device(f"cuda:{self.local_rank}" if dev.startswith("cuda") else dev)
        if dev.startswith("cuda") and os.environ.get("DPPO_SINGLE_DEVICE"):   # test rig: all ranks share cuda:0
            self.device = torch.device("cuda:0")
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.seed = cfg.get("seed", 42)
        random.seed(self.seed)
        np.random.seed(self.seed)
        torch.manual_seed(self.seed)
        self.use_wandb = False
        if cfg.get("wandb") is not None:
            log.info("wandb logging requested but disabled (no network on MI355X hosts); metrics go to result.pkl")

        # env batch: cfg.env.n_envs is the GLOBAL count, sharded evenly over ranks
        self.env_name = cfg.env.name
        self.n_envs_global = int(cfg.env.n_envs)
        self.n_envs, self.env_offset = shard_envs(self.n_envs_global, self.world_size, self.rank)
        wrappers = cfg.env.get("wrappers", None)
        self.venv = make_async(cfg.env.name, env_type=cfg.env.get("env_type", None), num_envs=self.n_envs,
                               asynchronous=True, max_episode_steps=cfg.env.max_episode_steps, wrappers=wrappers,
                               obs_dim=cfg.obs_dim, action_dim=cfg.action_dim, act_steps=cfg.act_steps,
                               obs_steps=cfg.cond_steps, family_seed=cfg.env.get("family_seed", 0),
                               native=bool(cfg.env.get("native", True)), synthetic=cfg.env.get("synthetic", False),
                               num_threads=cfg.env.get("num_threads", None),
                               sim_cost_us=float(cfg.env.get("sim_cost_us", 0.0)))
        self.venv.seed([self.seed + self.env_offset + i for i in range(self.n_envs)])  # train_agent.py:53-56
        self.n_cond_step = cfg.cond_steps
        self.obs_dim = cfg.obs_dim
        self.action_dim = cfg.action_dim
        self.act_steps = cfg.act_steps
        self.horizon_steps = cfg.horizon_steps
        self.max_episode_steps = cfg.env.max_episode_steps
        self.reset_at_iteration = cfg.env.get("reset_at_iteration", True)
        self.save_full_observations = cfg.env.get("save_full_observations", False)
        self.furniture_sparse_reward = False
        self.batch_size = int(cfg.train.batch_size)
        # data parallel: false (default) = the reference's PPO, global minibatch = batch_size rows
        # (batch_size / world per rank); true = batch_size rows PER RANK (a batch_size x world PPO)
        self.dp_scale_batch = bool(cfg.train.get("dp_scale_batch", False))

        self.model = instantiate(cfg.model, device=str(self.device), seed=self.seed)
        self.model.set_rng(self.seed, env_offset=self.env_offset)
        if self.world_size > 1:  # identical replicas (same seed already; broadcast guards against drift)
            for t in (self.model.base_params, self.model.train_params):
                broadcast_(t, src=0)
            self.model.repack()

        self.itr = 0
        self.n_train_itr = cfg.train.n_train_itr
        self.val_freq = cfg.train.val_freq
        self.force_train = cfg.train.get("force_train", False)
        self.n_steps = cfg.train.n_steps
        self.best_reward_threshold_for_success = cfg.env.get("best_reward_threshold_for_success", 3)
        self.max_grad_norm = cfg.train.get("max_grad_norm", None)

        self.logdir = cfg.get("logdir", "outputs")
        self.render_dir = os.path.join(self.logdir, "render")
        self.checkpoint_dir = os.path.join(self.logdir, "checkpoint")
        self.result_path = os.path.join(self.logdir, "result.pkl")
        if self.rank == 0:
            os.makedirs(self.checkpoint_dir, exist_ok=True)
        self.save_trajs = cfg.train.get("save_trajs", False)
        self.log_freq = cfg.train.get("log_freq", 1)
        self.save_model_freq = cfg.train.save_model_freq
        render = cfg.train.get("render", {}) or {}
        self.render_freq = render.get("freq", 1)
        self.n_render = render.get("num", 0)
        self.render_video = cfg.env.get("save_video", False)
        self.traj_plotter = None

    def run(self):
        pass

    def _ckpt_path(self, itr):
        # train_agent.py:127-142: state_{itr}.weights.h5 (Keras-3 layout, util/keras_weights.py);
        # train.checkpoint_format = npz keeps the .npz form
        ext = ".npz" if self.cfg.train.get("checkpoint_format", "h5") == "npz" else ".weights.h5"
        return os.path.join(self.checkpoint_dir, f"state_{itr}{ext}")

    def save_model(self):
        """train_agent.py:127-133."""
        if self.rank != 0:
            return
        path = self._ckpt_path(self.itr)
        self.model.save_weights(path)
        log.info("Saved model to %s", path)

    def load(self, itr):
        """train_agent.py:135-142. The file of train.checkpoint_format (default .weights.h5); a run saved
        in the other format is found too (npz was the default before round 2)."""
        path = self._ckpt_path(itr)
        if not os.path.exists(path):
            other = os.path.join(self.checkpoint_dir, f"state_{itr}" + (".weights.h5" if path.endswith(".npz") else ".npz"))
            if not os.path.exists(other):
                raise FileNotFoundError(f"no checkpoint for itr {itr}: neither {path} nor {other} exists "
                                        "(train.checkpoint_format selects h5 or npz for saving)")
            path = other
        self.model.load_weights(path)
        log.info("Loaded model from %s", path)

    def reset_env_all(self, verbose=False, options_venv=None, **kwargs):
        return self.venv.reset_arg(options_list=options_venv)

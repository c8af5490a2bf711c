"""DiffusionModel base (reference model/diffusion/diffusion.py:19-110): DDPM schedule buffers and
the shared configuration of the diffusion policy; standalone (the pretrain cfgs' `model`), it also
owns its network's parameters and the pretraining loss c_loss / p_losses / q_sample (:179-202)."""
import logging
import os
from collections import namedtuple

import numpy as np
import torch

from ... import ops
from ...util import keras_weights
from .sampling import ddim_buffers, ddpm_buffers

log = logging.getLogger(__name__)

Sample = namedtuple("Sample", "trajectories chains")


class DiffusionModel:
    def __init__(self, network, horizon_steps, obs_dim, action_dim, network_path=None, device="cuda:0",
                 denoised_clip_value=1.0, randn_clip_value=10.0, final_action_clip_value=None, eps_clip_value=None,
                 denoising_steps=100, predict_epsilon=True, use_ddim=False, ddim_discretize="uniform", ddim_steps=None,
                 precision="fp32", seed=42, ddim_eta=1.0, **kwargs):
        if not predict_epsilon:
            raise NotImplementedError("predict_epsilon=False is not used by the DPPO cfgs")
        if denoised_clip_value != 1.0:
            raise NotImplementedError("the sampler epilogue implements denoised_clip_value = 1.0 (diffusion.py:28)")
        if eps_clip_value is not None:
            # DDIM: the reference computes the clip and discards it (diffusion_vpg.py:213-214)
            log.info("eps_clip_value has no effect (the reference discards the clipped eps)")
        if precision not in ops._lib.PRECISION:
            raise ValueError(f"precision must be one of {sorted(ops._lib.PRECISION)}")
        self.device = torch.device(device)
        self.horizon_steps = horizon_steps
        self.obs_dim = obs_dim
        self.action_dim = action_dim
        self.denoising_steps = int(denoising_steps)
        self.predict_epsilon = predict_epsilon
        self.use_ddim = use_ddim
        self.ddim_steps = ddim_steps
        self.ddim_eta = float(ddim_eta)
        self.denoised_clip_value = denoised_clip_value
        self.final_action_clip_value = final_action_clip_value
        self.randn_clip_value = randn_clip_value
        self.eps_clip_value = eps_clip_value
        self.precision = precision
        self.seed = int(seed)
        self.network = network
        self.network_path = network_path
        buf = ddpm_buffers(self.denoising_steps)
        for k, v in buf.items():
            setattr(self, k, v)
        if use_ddim:
            # DDIM (BASELINE config 5): ddim_steps sampling rows at t = j K/S;
            # train/logprob use eta, eval (deterministic) sampling eta = 0 (diffusion_vpg.py:222-224)
            dd = ddim_buffers(self.denoising_steps, ddim_steps, ddim_eta)
            for k, v in dd.items():
                setattr(self, k, v)
            self.sampling_steps, self.time_stride = int(ddim_steps), dd["time_stride"]
            self.sched = torch.tensor(ops.sched_table(dd), device=self.device)
            self.sched_eval = torch.tensor(ops.sched_table(ddim_buffers(self.denoising_steps, ddim_steps, 0.0)),
                                           device=self.device)
        else:
            self.sampling_steps, self.time_stride = self.denoising_steps, 1
            self.sched = torch.tensor(ops.sched_table(buf), device=self.device)
            self.sched_eval = self.sched

    def sched_for(self, deterministic):
        """The schedule table of a sampling call (DDIM eval sampling runs eta = 0)."""
        return self.sched_eval if deterministic else self.sched

    # ------------------------------------------------------------------ pretraining (diffusion.py:179-202)
    def _pretrain_init(self):
        """Parameters of the standalone model's network (the pretrain cfgs: DiffusionMLP), packed for
        the row-tile kernels, on first use."""
        if getattr(self, "pre_dims", None) is not None:
            return
        net = self.network
        self.pre_dims = ops.ModelDims(obs_dim=self.obs_dim, action_dim=self.action_dim,
                                      horizon_steps=self.horizon_steps, cond_steps=net.cond_dim // self.obs_dim,
                                      time_dim=net.time_dim, actor_hidden=net.hidden,
                                      denoising_steps=self.denoising_steps, ft_denoising_steps=1, time_stride=1)
        self.pre_spec = ops.actor_param_spec(self.pre_dims)
        path = self.network_path
        if path is not None and not os.path.exists(str(path)):
            raise FileNotFoundError(f"network_path {str(path)!r} does not exist (null = seeded synthetic weights)")
        if path is not None and str(path).endswith(".npz"):
            with np.load(str(path), allow_pickle=False) as f:
                pref = "network." if any(k.startswith("network.") for k in f.files) else ""
                p = {n: np.asarray(f[pref + n], np.float32).reshape(s) for n, s in self.pre_spec}
        elif path is not None and str(path).endswith(".h5"):      # Keras-3 weights (util/keras_weights.py)
            p = keras_weights.load_actor(str(path), self.pre_spec)
        elif path is not None:
            raise ValueError(f"network_path {path}: .weights.h5 or .npz checkpoints")
        else:
            p = net.init_params(np.random.default_rng(self.seed))
        dev = self.device
        self.params = torch.tensor(ops.flatten_params(self.pre_spec, p), device=dev)
        self.pre_grads = torch.zeros_like(self.params)
        self.packed = ops.pack_actor(self.pre_dims, self.params, self.precision)
        # q_sample buffers and the DDPM table over all K training steps (DDIM only changes sampling)
        ddpm = ddpm_buffers(self.denoising_steps)
        self.q_sched = torch.tensor(ops.q_sched_table(ddpm), device=dev)
        self.pre_sched = torch.tensor(ops.sched_table(ddpm), device=dev)
        self.pre_metrics = torch.zeros(16, dtype=torch.float64, device=dev)
        self._pre_gen = torch.Generator(device=dev).manual_seed(self.seed)
        self._pre_ws, self._pre_ws_rows = None, 0

    def repack_network(self):
        """Re-derive the packed image after an optimiser step on self.params."""
        ops.pack_actor(self.pre_dims, self.params, self.precision, out=self.packed)

    def q_sample(self, x_start, t, noise):
        """diffusion.py:196-202 (device tensors, fp32 buffers)."""
        self._pretrain_init()
        q = self.q_sched[t.long()]
        shape = (-1,) + (1,) * (x_start.dim() - 1)
        return q[:, 0].reshape(shape) * x_start + q[:, 1].reshape(shape) * noise

    def p_losses(self, x_start, cond, t, noise=None, global_rows=None, loss_scale=1.0):
        """diffusion.py:186-194 (predict_epsilon): loss = mean((network(q_sample(x_0, t, noise), t, cond)
        - noise)^2) on the device; d loss / d params lands in self.pre_grads (dppo_pretrain_minibatch).
        x_start [B, Ta, Da] or [B, Ta*Da]; cond [B, To, Do] or a dict with "state"; t [B] int."""
        self._pretrain_init()
        d = self.pre_dims
        if isinstance(cond, dict):
            cond = cond["state"]
        B = x_start.shape[0]
        x0 = x_start.reshape(B, d.xd).to(self.device, torch.float32).contiguous()
        c = cond.reshape(B, d.sd).to(self.device, torch.float32).contiguous()
        t = t.to(self.device, torch.int32).contiguous()
        if noise is None:
            noise = torch.randn(B, d.xd, device=self.device, generator=self._pre_gen)
        noise = noise.reshape(B, d.xd).to(self.device, torch.float32).contiguous()
        if self._pre_ws is None or self._pre_ws_rows < B:
            self._pre_ws, self._pre_ws_rows = ops.ppo_workspace(d, self.precision, B, self.device), B
        return ops.pretrain_minibatch(d, self.precision, self.packed, self.params, self.pre_sched, self.q_sched, x0, c,
                                      t, noise, self._pre_ws, self.pre_grads, self.pre_metrics,
                                      global_rows=global_rows, loss_scale=loss_scale)

    def c_loss(self, actions, conditions, **kwargs):
        """diffusion.py:178-184: t ~ U{0, .., K-1} per sample (:182), then p_losses."""
        self._pretrain_init()
        B = actions.shape[0]
        t = torch.randint(0, self.denoising_steps, (B,), device=self.device, generator=self._pre_gen,
                          dtype=torch.int32)
        return self.p_losses(actions, conditions, t, **kwargs)

    def save_network(self, path):
        """The network alone: a Keras-3 weights file for *.h5 (the reference's
        self.model.network.save_weights, agent/pretrain/train_agent.py:150-154), else .npz."""
        params = ops.unflatten_params(self.pre_spec, self.params.detach().cpu().numpy())
        if str(path).endswith(".h5"):
            keras_weights.save_actor(str(path), params)
        else:
            np.savez(path, **{"network." + n: v for n, v in params.items()})

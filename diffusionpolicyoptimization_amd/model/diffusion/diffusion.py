"""DiffusionModel base (reference model/diffusion/diffusion.py:19-110): DDPM schedule buffers and
the shared configuration of the diffusion policy."""
import logging
from collections import namedtuple

import numpy as np
import torch

from ... import ops
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

"""CriticObs (reference model/common/critic.py:15-54): ResidualMLP([Do*To, h, h, h, 1], Mish).

Construction mirrors the reference kwargs; the forward runs the HIP value kernel
(dppo_critic_forward) once the owning VPGDiffusion has placed the weights on the device."""
import numpy as np
import torch

from .mlp import ResidualMLP


class CriticObs:
    def __init__(self, cond_dim, mlp_dims, activation_type="Mish", use_layernorm=False, residual_style=False,
                 **kwargs):
        if not residual_style:
            raise NotImplementedError("CriticObs(residual_style=False) is not implemented on MI355X")
        if activation_type != "Mish":
            raise NotImplementedError("the critic kernels implement the cfg's Mish activation")
        self.cond_dim = cond_dim
        self.net = ResidualMLP([cond_dim] + list(mlp_dims) + [1], activation_type=activation_type,
                               use_layernorm=use_layernorm)
        self.hidden = self.net.hidden
        self._owner = None

    def init_params(self, rng):
        return self.net.init_params(rng)

    def __call__(self, cond):
        """cond: {"state": [B, To, Do]} or [B, To*Do] -> values [B, 1] (device tensor)."""
        if self._owner is None:
            raise RuntimeError("CriticObs has no device weights yet (construct it through PPODiffusion)")
        return self._owner.critic_values(cond)[:, None]

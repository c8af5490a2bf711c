"""DiffusionMLP (reference model/diffusion/mlp_diffusion.py:12-90).

input = concat[x.flat (Ta*Da), t_emb (time_dim), state.flat (To*Do)] -> ResidualMLP -> eps, with
t_emb = Dense(2*time_dim, mish)(SinusoidalPosEmb(t)) -> Dense(time_dim). The network is evaluated
only inside the fused HIP kernels (sampler / logprob / PPO update), so this class is the
configuration + parameter container."""
import numpy as np

from ..common.mlp import ResidualMLP, glorot_uniform


class DiffusionMLP:
    def __init__(self, action_dim, horizon_steps, cond_dim, time_dim=16, mlp_dims=(256, 256), cond_mlp_dims=None,
                 activation_type="Mish", out_activation_type="Identity", use_layernorm=False, residual_style=False):
        if cond_mlp_dims is not None:
            raise NotImplementedError("cond_mlp_dims (obs encoder) is not used by the gym fine-tune cfgs")
        if not residual_style:
            raise NotImplementedError("DiffusionMLP(residual_style=False) is not implemented on MI355X")
        if activation_type != "ReLU":
            raise NotImplementedError("the actor kernels implement the cfg's ReLU activation")
        self.action_dim, self.horizon_steps, self.cond_dim, self.time_dim = action_dim, horizon_steps, cond_dim, time_dim
        self.mlp_dims = list(mlp_dims)
        self.activation_type = activation_type
        self.out_activation_type = out_activation_type
        self.residual_style = residual_style
        output_dim = action_dim * horizon_steps
        self.input_dim = time_dim + output_dim + cond_dim
        self.mlp_mean = ResidualMLP([self.input_dim] + self.mlp_dims + [output_dim], activation_type=activation_type,
                                    out_activation_type=out_activation_type, use_layernorm=use_layernorm)
        self.hidden = self.mlp_mean.hidden

    def init_params(self, rng):
        td = self.time_dim
        p = {"time_w1": glorot_uniform(rng, td, 2 * td), "time_b1": np.zeros(2 * td, np.float32),
             "time_w2": glorot_uniform(rng, 2 * td, td), "time_b2": np.zeros(td, np.float32)}
        p.update(self.mlp_mean.init_params(rng))
        return p

    def get_config(self):
        return dict(action_dim=self.action_dim, horizon_steps=self.horizon_steps, cond_dim=self.cond_dim,
                    time_dim=self.time_dim, mlp_dims=self.mlp_dims, cond_mlp_dims=None,
                    activation_type=self.activation_type, out_activation_type=self.out_activation_type,
                    use_layernorm=False, residual_style=self.residual_style)

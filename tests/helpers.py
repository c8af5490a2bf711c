"""Shared fixtures for the parity tests: seeded synthetic weights and inputs."""
import numpy as np

from oracle import dppo_oracle as O

HOPPER = dict(obs_dim=11, action_dim=3, horizon_steps=4, cond_steps=1, time_dim=16, actor_hidden=512,
              critic_hidden=256, denoising_steps=20, ft_denoising_steps=10)
WALKER = dict(HOPPER, obs_dim=17, action_dim=6)
# an action width the kernels do not specialise (XD = 8: padded to the generic 32-wide instantiation)
NARROW = dict(HOPPER, action_dim=2)
# BASELINE config 5: DDIM, 10 sampling rows over K = 20 (time stride 2), all fine-tuned
HOPPER_DDIM = dict(HOPPER, denoising_steps=10, ft_denoising_steps=10, time_stride=2)


def make_models(seed=0, dims=HOPPER, bias_scale=0.05, ft_perturb=0.02):
    rng = np.random.default_rng(seed)
    base = O.init_actor(rng, dims["obs_dim"], dims["action_dim"], dims["horizon_steps"], dims["cond_steps"],
                        dims["time_dim"], dims["actor_hidden"], bias_scale=bias_scale)
    ft = {k: (v + rng.normal(0, ft_perturb, v.shape).astype(np.float32)) for k, v in base.items()}
    critic = O.init_critic(rng, dims["obs_dim"], dims["cond_steps"], dims["critic_hidden"], bias_scale=bias_scale)
    return base, ft, critic


def to_f64(p):
    return {k: np.asarray(v, np.float64) for k, v in p.items()}

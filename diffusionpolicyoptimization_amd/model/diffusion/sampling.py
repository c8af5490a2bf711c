"""Host-side DDPM schedule buffers (model/diffusion/sampling.py:7-29 and diffusion.py:57-73 of the
reference). Computed once at model construction in fp32, exactly as the TF buffers are, and
uploaded as the [K][8] table the kernels read (include/dppo.h, DPPO_SCHED_COLS)."""
import numpy as np


def cosine_beta_schedule(timesteps, s=0.008, dtype=np.float32):
    """sampling.py:7-17. Note the reference's linspace(0, K+1, K+1) grid (spacing (K+1)/K)."""
    n = timesteps + 1
    grid = np.linspace(0, n, n)
    abar = np.cos(((grid / n) + s) / (1 + s) * np.pi * 0.5) ** 2
    abar = abar / abar[0]
    return np.clip(1 - abar[1:] / abar[:-1], 0, 0.999).astype(dtype)


def ddpm_buffers(denoising_steps):
    """diffusion.py:57-73, fp32 arithmetic like the tf.float32 buffers."""
    one = np.float32(1.0)
    betas = cosine_beta_schedule(denoising_steps)
    alphas = (one - betas).astype(np.float32)
    abar = np.cumprod(alphas, dtype=np.float32)
    abar_prev = np.concatenate([np.ones(1, np.float32), abar[:-1]]).astype(np.float32)
    var = (betas * (one - abar_prev) / (one - abar)).astype(np.float32)
    return {
        "betas": betas,
        "alphas": alphas,
        "alphas_cumprod": abar,
        "alphas_cumprod_prev": abar_prev,
        "sqrt_recip_alphas_cumprod": np.sqrt(one / abar).astype(np.float32),
        "sqrt_recipm1_alphas_cumprod": np.sqrt(one / abar - one).astype(np.float32),
        "ddpm_var": var,
        "ddpm_logvar_clipped": np.log(np.clip(var, np.float32(1e-20), np.inf)).astype(np.float32),
        "ddpm_mu_coef1": (betas * np.sqrt(abar_prev) / (one - abar)).astype(np.float32),
        "ddpm_mu_coef2": ((one - abar_prev) * np.sqrt(alphas) / (one - abar)).astype(np.float32),
    }


def extract(a, t, x_shape):
    """sampling.py:20-24: gather a[t] and reshape to [B, 1, ...]."""
    t = np.asarray(t)
    return np.asarray(a)[t].reshape((t.shape[0],) + (1,) * (len(x_shape) - 1))


def make_timesteps(batch_size, i):
    """sampling.py:27-29."""
    return np.full((batch_size,), i, dtype=np.int64)

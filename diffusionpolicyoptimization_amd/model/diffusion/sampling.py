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


def ddim_buffers(denoising_steps, ddim_steps, eta=1.0):
    """DDIM sub-sequence buffers (diffusion.py:76-96) in fp32, following the documented formulas
    (diffusion_vpg.py:184-234) with the corrections SURVEY.md §8 quirk 6 lists: the sub-sequence is
    walked from its largest t down, alpha_prev is the previous element OF THE SUB-SEQUENCE, eta is
    a fixed number (EtaFixed; eta = 0 is the deterministic/eval schedule), and eps is recomputed
    from the clipped x0. Row j (j = 0..S-1, diffusion time t = j * K/S) is the sampling row the
    kernels index like a DDPM t; the affine coefficients of the schedule table (include/dppo.h):
        x0 = c0 x - c1 eps, clipped;  eps' = (x - sqrt(abar) x0) / sqrt(1 - abar)
        mu = sqrt(abar_prev) x0 + d eps'  =  c2 x0 + c3 x
    """
    if ddim_steps is None or ddim_steps < 1 or denoising_steps % ddim_steps:
        raise ValueError(f"ddim_steps must divide denoising_steps ({denoising_steps}), got {ddim_steps}")
    f = np.float32
    one = f(1.0)
    ratio = denoising_steps // ddim_steps
    abar_all = ddpm_buffers(denoising_steps)["alphas_cumprod"]
    ddim_t = np.arange(ddim_steps) * ratio                           # uniform discretisation (:80-82)
    a = abar_all[ddim_t].astype(f)
    a_prev = np.concatenate([np.ones(1, f), a[:-1]]).astype(f)      # corrected: previous sub-sequence element
    sfac = np.sqrt((one - a_prev) / (one - a) * (one - a / a_prev)).astype(f)   # sigma / eta, unclamped
    sig = (f(eta) * sfac).astype(f)
    sig = np.maximum(sig, f(1e-10))                                   # .clamp_(min=1e-10) (:228)
    d = np.sqrt(np.clip(one - a_prev - sig * sig, f(0.0), f(1e6))).astype(f)
    sa, s1a = np.sqrt(a).astype(f), np.sqrt(one - a).astype(f)
    return {
        "ddim_t": ddim_t, "ddim_alphas": a, "ddim_alphas_prev": a_prev, "ddim_sigmas": sig, "ddim_eta": float(eta),
        "ddim_c0": (one / sa).astype(f),
        "ddim_c1": (s1a / sa).astype(f),
        "ddim_c2": (np.sqrt(a_prev) - d * sa / s1a).astype(f),
        "ddim_c3": (d / s1a).astype(f),
        "ddim_logvar": np.log(sig * sig).astype(f),
        "ddim_sfac": sfac,
        "ddim_sqrt_alphas_prev": np.sqrt(a_prev).astype(f), "ddim_sqrt_alphas": sa, "ddim_sqrt_1m_alphas": s1a,
        "time_stride": ratio,
    }


def extract(a, t, x_shape):
    """sampling.py:20-24: gather a[t] and reshape to [B, 1, ...]."""
    t = np.asarray(t)
    return np.asarray(a)[t].reshape((t.shape[0],) + (1,) * (len(x_shape) - 1))


def make_timesteps(batch_size, i):
    """sampling.py:27-29."""
    return np.full((batch_size,), i, dtype=np.int64)

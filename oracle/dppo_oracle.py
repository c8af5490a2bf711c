"""Float64 NumPy restatement of the DPPO fine-tuning hot path of the TF reference.

TEST INFRASTRUCTURE ONLY — this module is the parity checker. It may be imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product package
(diffusionpolicyoptimization_amd) never imports it and fails loudly without its HIP
library.

Every function cites the reference file:line (relative to the reference repo root) whose
semantics it restates. Weights use the Keras layout (kernel [in, out], bias [out]).

Parity pinning:
  * reward scaling is pinned bit-for-bit against the reference's own util/reward_scaling.py
    (importable in the build container) through tests/golden/reward_scaling.npz;
  * the cosine schedule is pinned against SURVEY.md §8(a)-a1's fp32 golden values;
  * everything downstream of TensorFlow / Keras / TF-Probability (Dense, mish, Normal.log_prob,
    AdamW) is "parity unpinned" at the TF boundary: no reference test or fixture exists and
    TF is not installable, so the restatement follows the cited formulas.
"""
import math

import numpy as np

LOG_2PI_HALF = 0.5 * math.log(2.0 * math.pi)


# ----------------------------------------------------------------------------------------------
# a1/a2: schedule (model/diffusion/sampling.py:7-17, model/diffusion/diffusion.py:57-73)
# ----------------------------------------------------------------------------------------------
def cosine_beta_schedule(K, s=0.008):
    """sampling.py:7-17 — note linspace(0, K+1, K+1) (spacing (K+1)/K), cast to fp32."""
    steps = K + 1
    x = np.linspace(0, steps, steps)
    ac = np.cos(((x / steps) + s) / (1 + s) * np.pi * 0.5) ** 2
    ac = ac / ac[0]
    betas = 1 - (ac[1:] / ac[:-1])
    return np.clip(betas, 0, 0.999).astype(np.float32)


def ddpm_schedule(K):
    """diffusion.py:57-73 computed in fp32 like the TF buffers. Returns dict of fp32 [K]."""
    f = np.float32
    betas = cosine_beta_schedule(K)
    alphas = (f(1.0) - betas).astype(np.float32)
    ac = np.cumprod(alphas, dtype=np.float32)  # tf.math.cumprod in fp32
    ac_prev = np.concatenate([np.ones(1, np.float32), ac[:-1]]).astype(np.float32)
    sqrt_recip = np.sqrt(f(1.0) / ac).astype(np.float32)
    sqrt_recipm1 = np.sqrt(f(1.0) / ac - f(1.0)).astype(np.float32)
    var = (betas * (f(1.0) - ac_prev) / (f(1.0) - ac)).astype(np.float32)
    logvar = np.log(np.clip(var, f(1e-20), np.inf)).astype(np.float32)
    coef1 = (betas * np.sqrt(ac_prev) / (f(1.0) - ac)).astype(np.float32)
    coef2 = ((f(1.0) - ac_prev) * np.sqrt(alphas) / (f(1.0) - ac)).astype(np.float32)
    return dict(betas=betas, alphas=alphas, alphas_cumprod=ac, alphas_cumprod_prev=ac_prev,
                sqrt_recip_alphas_cumprod=sqrt_recip, sqrt_recipm1_alphas_cumprod=sqrt_recipm1,
                ddpm_var=var, ddpm_logvar_clipped=logvar, ddpm_mu_coef1=coef1, ddpm_mu_coef2=coef2)


def ddim_schedule(K, S, eta=1.0, dtype=np.float32):
    """DDIM sub-sequence (diffusion.py:76-96; diffusion_vpg.py:184-234 documented formulas) with
    the corrections of SURVEY.md §8 quirk 6: walked from the largest t down, alpha_prev = the
    previous SUB-SEQUENCE element, fixed eta, eps recomputed from the clipped x0. PARITY
    UNPINNED: the reference DDIM path cannot run (quirk 6), so this restates the formulas.
    Returns the affine per-row coefficients under the DDPM keys p_mean_var reads (row j = DDIM
    index, diffusion time j*K/S), plus the raw sub-sequence arrays (p_mean_var_ddim_direct)."""
    f = dtype
    one = f(1.0)
    ratio = K // S
    ac = ddpm_schedule(K)["alphas_cumprod"]
    a = ac[np.arange(S) * ratio].astype(f)
    ap = np.concatenate([np.ones(1, f), a[:-1]]).astype(f)
    sfac = np.sqrt((one - ap) / (one - a) * (one - a / ap)).astype(f)   # sigma / eta before the clamp
    sig = np.maximum((f(eta) * sfac).astype(f), f(1e-10))
    d = np.sqrt(np.clip(one - ap - sig * sig, 0, 1e6)).astype(f)
    sa, s1a = np.sqrt(a).astype(f), np.sqrt(one - a).astype(f)
    return dict(sqrt_recip_alphas_cumprod=(one / sa).astype(f), sqrt_recipm1_alphas_cumprod=(s1a / sa).astype(f),
                ddpm_mu_coef1=(np.sqrt(ap) - d * sa / s1a).astype(f), ddpm_mu_coef2=(d / s1a).astype(f),
                ddpm_logvar_clipped=np.log(sig * sig).astype(f), time_stride=ratio, eval_floor=0.0,
                eval_zero=np.ones(S, bool), ddim_alphas=a, ddim_alphas_prev=ap, ddim_sigmas=sig, ddim_dir=d,
                ddim_sfac=sfac, ddim_eta=float(eta))


# ----------------------------------------------------------------------------------------------
# §8(f) row 4: a learnable DDIM eta. The reference builds VPGDiffusion(eta=..., learn_eta=...) and an
# eta AdamW (train_ppo_diffusion_agent.py:28-45) but its eta module (model/diffusion/eta.py of the
# original DPPO) is absent and the eta step is commented out (:358-359): PARITY UNPINNED. Restated
# from the original DPPO's EtaFixed: eta = min + (max - min) (tanh(logit) + 1) / 2, one scalar for
# every row, entering p_mean_var through sigma = eta s_t and the direction coefficient
# d = sqrt(clip(1 - abar_prev - sigma^2, 0, 1e6)) (diffusion_vpg.py:219-234).
# ----------------------------------------------------------------------------------------------
def eta_from_logit(logit, eta_min, eta_max):
    return eta_min + (eta_max - eta_min) * 0.5 * (math.tanh(logit) + 1.0)


def eta_logit_init(base_eta, eta_min, eta_max):
    """EtaFixed's initial logit: atanh(2 (base - min) / (max - min) - 1)."""
    return math.atanh(2.0 * (base_eta - eta_min) / (eta_max - eta_min) - 1.0)


def ddim_eta_grad_terms(sched, t, eta, min_logprob_std):
    """Per-row derivatives of the DDIM row's direction coefficient d and log-prob std w.r.t. eta
    (zero where a clamp or clip holds the value): dd/deta = -sigma s / d, dstd/deta = s."""
    s = sched["ddim_sfac"].astype(np.float64)[t]
    sig_raw = eta * s
    sig = np.maximum(sig_raw, 1e-10)
    inner = 1.0 - sched["ddim_alphas_prev"].astype(np.float64)[t] - sig ** 2
    dd = np.where((inner > 0) & (inner < 1e6) & (sig_raw > 1e-10),
                  -sig * s / np.sqrt(np.maximum(inner, 1e-300)), 0.0)
    dstd = np.where((sig_raw > 1e-10) & (sig > min_logprob_std) & (sig < 1e6), s, 0.0)
    return dd, dstd


def p_mean_var_ddim_direct(sched, eps, x, j, denoised_clip=1.0):
    """The documented DDIM mean, term by term (diffusion_vpg.py:193-196, 204-212, 221-232):
    x0 = (x - sqrt(1-a) eps)/sqrt(a); clip; eps = (x - sqrt(a) x0)/sqrt(1-a);
    mu = sqrt(a_prev) x0 + sqrt(1 - a_prev - sigma^2) eps."""
    sh = (-1,) + (1,) * (x.ndim - 1)
    a = sched["ddim_alphas"].astype(np.float64)[j].reshape(sh)
    ap = sched["ddim_alphas_prev"].astype(np.float64)[j].reshape(sh)
    sig = sched["ddim_sigmas"].astype(np.float64)[j].reshape(sh)
    x0 = np.clip((x - np.sqrt(1 - a) * eps) / np.sqrt(a), -denoised_clip, denoised_clip)
    e2 = (x - np.sqrt(a) * x0) / np.sqrt(1 - a)
    mu = np.sqrt(ap) * x0 + np.sqrt(np.clip(1 - ap - sig ** 2, 0, 1e6)) * e2
    return mu, np.log(sig ** 2)


def _tstride(sched):
    return int(sched.get("time_stride", 1))


# ----------------------------------------------------------------------------------------------
# activations (model/common/mlp.py:6-14) and Dense
# ----------------------------------------------------------------------------------------------
def relu(x):
    return np.maximum(x, 0.0)


def relu_grad(h):
    return (h > 0).astype(np.float64)


def softplus(x):
    return np.logaddexp(0.0, x)


def mish(x):
    """keras.activations.mish: x * tanh(softplus(x))."""
    return x * np.tanh(softplus(x))


def mish_grad(x):
    sp = softplus(x)
    th = np.tanh(sp)
    sig = 1.0 / (1.0 + np.exp(-x))
    return th + x * (1.0 - th * th) * sig


ACT = {"ReLU": (relu, relu_grad), "Mish": (mish, mish_grad)}


def dense(x, w, b):
    return x @ np.asarray(w, np.float64) + np.asarray(b, np.float64)


# ----------------------------------------------------------------------------------------------
# a3: SinusoidalPosEmb (model/diffusion/modules.py:4-15)
# ----------------------------------------------------------------------------------------------
def sinusoidal_pos_emb(t, dim=16):
    half = dim // 2
    emb = math.log(10000) / (half - 1)
    freqs = np.exp(np.arange(half, dtype=np.float64) * -emb)
    e = np.asarray(t, np.float64)[:, None] * freqs[None, :]
    return np.concatenate([np.sin(e), np.cos(e)], axis=-1)


# ----------------------------------------------------------------------------------------------
# a5: ResidualMLP with one TwoLayerPreActivationResNetLinear block (model/common/mlp.py:95-206)
#   h1 = x W_in + b_in ; h2 = act(h1) W_1 + b_1 ; h3 = act(h2) W_2 + b_2 + h1 ; y = h3 W_out + b_out
# ----------------------------------------------------------------------------------------------
def round_bf16(x):
    """fp32 -> bf16 round-to-nearest-even -> back (what v_cvt_pk_bf16_f32 does on gfx950)."""
    u = np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32).astype(np.uint64)
    u = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def round_fp16(x):
    """fp32 -> fp16 round-to-nearest-even -> back (v_cvt_pk_f16_f32; the fp16 operand policy)."""
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float64)


FP16_GRAD_SCALE = 4096.0


def fp16_grad_scale(global_rows):
    """dppo_grad_scale_rows (csrc/dppo_internal.h): the largest power of two <= min(4096, rows),
    so a per-row gradient image (g / rows) times the scale stays <= |g| and cannot overflow."""
    s = 1.0
    while s < FP16_GRAD_SCALE and 2 * s <= global_rows:
        s *= 2.0
    return s


def round_fp16_rows(global_rows):
    """round_fp16 whose gradient images use the row-tied scale of a global_rows minibatch."""
    sc = fp16_grad_scale(global_rows)

    def rnd(x):
        return round_fp16(x)
    rnd.grad_round = lambda x: round_fp16(np.asarray(x, np.float64) * sc) / sc
    return rnd


def _round_fp16_grad(x):
    """The fp16 kernels store backward images as fp16(GRAD_SCALE * g) (PolicyF16, dppo_common.cuh)."""
    return round_fp16(np.asarray(x, np.float64) * FP16_GRAD_SCALE) / FP16_GRAD_SCALE


round_fp16.grad_round = _round_fp16_grad


def _ident(x):
    return np.asarray(x, np.float64)


def residual_mlp_forward(p, x, act, prefix, rnd=None, round_h3=True):
    """rnd: optional operand-rounding function applied exactly where the bf16 kernels round
    (GEMM A/B operands; accumulators, residual h1 and epilogues stay fp32). None = exact f64.
    round_h3=False: the out-Dense input is not rounded (the split sampler feeds it as a hi/lo
    bf16 pair, sampler_split.hip), only its weights are. It is also the folded form of the actor's
    row tiles (csrc/rowtile.hip, dppo_layout.h RT_*: eps = relu(h2) M + a0 M0 + b with M = rnd(W_l2)
    rnd(W_out), M0 = rnd(W_in) rnd(W_out) to fp32), whose backward forms d relu(h2) = dy M^T without
    rounding dh3 (residual_mlp_backward reads cache["fold"])."""
    a, _ = ACT[act]
    R = rnd or _ident
    xr = R(x)
    h1 = xr @ R(p[prefix + "in_w"]) + np.asarray(p[prefix + "in_b"], np.float64)
    u1 = R(a(h1))
    h2 = u1 @ R(p[prefix + "l1_w"]) + np.asarray(p[prefix + "l1_b"], np.float64)
    u2 = R(a(h2))
    h3 = u2 @ R(p[prefix + "l2_w"]) + np.asarray(p[prefix + "l2_b"], np.float64) + h1
    h3r = R(h3) if round_h3 else np.asarray(h3, np.float64)
    y = h3r @ R(p[prefix + "out_w"]) + np.asarray(p[prefix + "out_b"], np.float64)
    return y, dict(x=xr, h1=h1, u1=u1, h2=h2, u2=u2, h3=h3r, R=R, fold=not round_h3)


def residual_mlp_backward(p, cache, dy, act, prefix):
    """Returns (grads dict, dx). dx uses the unrounded input weights (the kernels form d t_emb
    from fp32 parameters)."""
    _, ag = ACT[act]
    R = cache.get("R", _ident)
    Rg = getattr(R, "grad_round", R)        # rounding of the gradient images (fp16: scaled)
    g = {}
    dyr = Rg(dy)
    g[prefix + "out_w"] = cache["h3"].T @ dyr
    g[prefix + "out_b"] = dyr.sum(0)
    wo = R(p[prefix + "out_w"])
    dh3 = dyr @ wo.T
    dh3r = Rg(dh3)
    # l2's weight gradient through the linear out layer (the kernels form no dh3 image for it,
    # csrc/update.hip l2_back_rows): u2^T (dy W_out^T) = (u2^T dy) W_out^T, unrounded dh3
    g[prefix + "l2_w"] = (cache["u2"].T @ dyr) @ wo.T
    g[prefix + "l2_b"] = g[prefix + "out_b"] @ wo.T
    if cache.get("fold"):   # the folded row tile: dy (R(W_l2) R(W_out))^T, dh3 unrounded on this path
        du2 = dyr @ (R(p[prefix + "l2_w"]) @ wo).T
    else:
        du2 = dh3r @ R(p[prefix + "l2_w"]).T
    dh2 = Rg(du2 * ag(cache["h2"]))
    g[prefix + "l1_w"] = cache["u1"].T @ dh2
    g[prefix + "l1_b"] = dh2.sum(0)
    du1 = dh2 @ R(p[prefix + "l1_w"]).T
    dh1 = Rg(dh3r + du1 * ag(cache["h1"]))   # the kernels re-read dh3 from its (rounded) LDS tile
    g[prefix + "in_w"] = cache["x"].T @ dh1
    g[prefix + "in_b"] = dh1.sum(0)
    dx = dh1 @ np.asarray(p[prefix + "in_w"], np.float64).T
    return g, dx


# ----------------------------------------------------------------------------------------------
# a4: DiffusionMLP (model/diffusion/mlp_diffusion.py:38-90); time MLP Dense(16->32, mish)->Dense(32->16)
# ----------------------------------------------------------------------------------------------
def time_mlp_forward(p, t, time_dim=16):
    e = sinusoidal_pos_emb(t, time_dim)
    a1 = dense(e, p["time_w1"], p["time_b1"])
    m1 = mish(a1)
    temb = dense(m1, p["time_w2"], p["time_b2"])
    return temb, dict(e=e, a1=a1, m1=m1)


def time_mlp_backward(p, cache, dtemb):
    g = {"time_w2": cache["m1"].T @ dtemb, "time_b2": dtemb.sum(0)}
    dm1 = dtemb @ np.asarray(p["time_w2"], np.float64).T
    da1 = dm1 * mish_grad(cache["a1"])
    g["time_w1"] = cache["e"].T @ da1
    g["time_b1"] = da1.sum(0)
    return g


def diffusion_mlp_forward(p, x, t, state, act="ReLU", rnd=None, round_h3=True):
    """x [B,Ta,Da], t [B] int, state [B,To,Do] -> eps [B,Ta,Da]; cond concat [x, t_emb, state] (:86)."""
    B = x.shape[0]
    temb, tcache = time_mlp_forward(p, t)
    inp = np.concatenate([x.reshape(B, -1), temb, state.reshape(B, -1)], axis=-1).astype(np.float64)
    y, cache = residual_mlp_forward(p, inp, act, "", rnd, round_h3)
    cache["time"] = tcache
    cache["t"] = np.asarray(t)
    return y.reshape(x.shape), cache


def diffusion_mlp_backward(p, cache, deps, xdim, act="ReLU"):
    B = deps.shape[0]
    g, dinp = residual_mlp_backward(p, cache, deps.reshape(B, -1), act, "")
    tdim = p["time_w2"].shape[1]
    dtemb = dinp[:, xdim:xdim + tdim]
    g.update(time_mlp_backward(p, cache["time"], dtemb))
    return g


# ----------------------------------------------------------------------------------------------
# a6: CriticObs (model/common/critic.py:15-54): ResidualMLP([Do,256,256,256,1], Mish)
# ----------------------------------------------------------------------------------------------
def critic_forward(pc, state, act="Mish", rnd=None):
    B = state.shape[0]
    v, cache = residual_mlp_forward(pc, state.reshape(B, -1).astype(np.float64), act, "", rnd)
    return v, cache


# ----------------------------------------------------------------------------------------------
# a8: p_mean_var, DDPM branch (model/diffusion/diffusion_vpg.py:152-245)
# ----------------------------------------------------------------------------------------------
def p_mean_var(sched, eps, x, t, denoised_clip=1.0):
    t = np.asarray(t)
    sh = (-1,) + (1,) * (x.ndim - 1)
    c1 = sched["sqrt_recip_alphas_cumprod"].astype(np.float64)[t].reshape(sh)
    c2 = sched["sqrt_recipm1_alphas_cumprod"].astype(np.float64)[t].reshape(sh)
    xr = c1 * x - c2 * eps                                       # :198-201
    unclipped = np.abs(xr) <= denoised_clip
    xr = np.clip(xr, -denoised_clip, denoised_clip)              # :204-206
    m1 = sched["ddpm_mu_coef1"].astype(np.float64)[t].reshape(sh)
    m2 = sched["ddpm_mu_coef2"].astype(np.float64)[t].reshape(sh)
    mu = m1 * xr + m2 * x                                        # :239-242
    logvar = sched["ddpm_logvar_clipped"].astype(np.float64)[t].reshape(sh)
    return mu, logvar, dict(m1=m1, c1=c1, c2=c2, unclipped=unclipped)


# ----------------------------------------------------------------------------------------------
# a9: sampler VPGDiffusion.call (diffusion_vpg.py:250-339), DDPM, with injected noise
# ----------------------------------------------------------------------------------------------
def sample(p_base, p_ft, sched, state, x_T, z, ft_steps, deterministic=False, min_std=0.1,
           randn_clip=3.0, final_clip=None, rnd=None, round_h3=True):
    """state [E,To,Do]; x_T [E,Ta,Da]; z [K,E,Ta,Da] raw N(0,1) draws for loop index i (t=K-1-i).
    Returns (trajectories [E,Ta,Da], chains [E,K'+1,Ta,Da]). round_h3: see residual_mlp_forward."""
    K = z.shape[0]
    x = np.asarray(x_T, np.float64)
    chain = []
    if ft_steps == K:
        chain.append(x.copy())                                   # :286-287
    for i in range(K):
        t = K - 1 - i
        tb = np.full(x.shape[0], t)
        params = p_ft if t < ft_steps else p_base                # :161-180
        eps, _ = diffusion_mlp_forward(params, x, tb * _tstride(sched), state, rnd=rnd, round_h3=round_h3)
        mu, logvar, _ = p_mean_var(sched, eps, x, tb)
        std = np.exp(0.5 * logvar)                               # :301
        ez = sched["eval_zero"][t] if "eval_zero" in sched else t == 0
        if deterministic and ez:                                 # :303-315 (DDIM: always 0)
            std = np.zeros_like(std)
        elif deterministic:
            std = np.clip(std, sched.get("eval_floor", 1e-3), 1e6)
        else:
            std = np.clip(std, min_std, 1e6)
        noise = np.clip(z[i], -randn_clip, randn_clip)           # :319
        x = mu + std * noise                                     # :320
        if final_clip is not None and i == K - 1:                # :323-327
            x = np.clip(x, -final_clip, final_clip)
        if t <= ft_steps:                                        # :330-331
            chain.append(x.copy())
    return x, np.stack(chain, axis=1)


def bc_loss(p_base, p_ft, sched, state, x_T, z, ft_steps, min_std=0.1, randn_clip=3.0, min_logprob_std=0.1,
            rnd=None):
    """c_loss's behaviour-cloning term (diffusion_ppo.py:63-71): chains of the base policy for every
    denoising step (use_base_policy=True, diffusion_vpg.py:175-176), their log-probs under actor_ft,
    clipped to [-5, 2]; -mean over every element. Reported only (agent :340-342)."""
    _, chains = sample(p_base, p_base, sched, state, x_T, z, ft_steps, min_std=min_std, randn_clip=randn_clip,
                       rnd=rnd, round_h3=False)
    lp = get_logprobs(p_ft, sched, state, chains, ft_steps, min_logprob_std=min_logprob_std, rnd=rnd)
    return -float(np.clip(lp, -5.0, 2.0).mean())


def gaussian_logprob(x, mu, std):
    """tfp Normal(mu, std).log_prob(x) (diffusion_vpg.py:419-422)."""
    return -0.5 * ((x - mu) / std) ** 2 - np.log(std) - LOG_2PI_HALF


# ----------------------------------------------------------------------------------------------
# a10: get_logprobs (diffusion_vpg.py:343-425)
# ----------------------------------------------------------------------------------------------
def get_logprobs(p_ft, sched, state, chains, ft_steps, min_logprob_std=0.1, rnd=None, round_h3=False):
    """state [n,To,Do], chains [n,K'+1,Ta,Da] -> logprob [n*K', Ta, Da]; row = n*K' + j, t = K'-1-j.
    round_h3=False: the folded row tile's rounding points (residual_mlp_forward)."""
    n = chains.shape[0]
    cond = np.repeat(state, ft_steps, axis=0)                    # :374-379 (sample-major tile)
    t_all = np.tile(np.arange(ft_steps - 1, -1, -1), n)          # :385-390
    prev = chains[:, :-1].reshape(-1, *chains.shape[2:])          # :402-407
    nxt = chains[:, 1:].reshape(-1, *chains.shape[2:])
    eps, _ = diffusion_mlp_forward(p_ft, prev, t_all * _tstride(sched), cond, rnd=rnd, round_h3=round_h3)
    mu, logvar, _ = p_mean_var(sched, eps, prev, t_all)
    std = np.clip(np.exp(0.5 * logvar), min_logprob_std, 1e6)    # :417-418
    return gaussian_logprob(nxt, mu, std)


# ----------------------------------------------------------------------------------------------
# a11 + a12: get_logprobs_subsample + PPODiffusion.c_loss and its gradient
#   (diffusion_vpg.py:427-481, diffusion_ppo.py:32-132, train_ppo_diffusion_agent.py:340)
# ----------------------------------------------------------------------------------------------
def c_loss(p_ft, pc, sched, obs, chains_prev, chains_next, denoising_inds, returns, oldvalues,
           advantages, oldlogprobs, ft_steps, gamma_denoising=0.99, clip_ploss_coef=0.01,
           clip_ploss_coef_base=0.01, clip_ploss_coef_rate=3.0, clip_vloss_coef=None,
           norm_adv=True, min_logprob_std=0.1, vf_coef=0.5, with_grad=True, reward_horizon=4, rnd=None,
           adv_mean_std=None, denom=None, critic_dedup=None, eta_grad=False, round_h3=False):
    """Returns (metrics dict, grads_actor dict, grads_critic dict).

    Data-parallel restatement hooks: adv_mean_std overrides the minibatch
    advantage mean/std (the global ones), denom overrides the row count the means divide by
    (the global minibatch size) — summing such per-shard gradients gives the full-batch one.
    round_h3=False: the folded actor row tile's rounding points (residual_mlp_forward).

    oldlogprobs may be per element [b,Ta,Da] (clipped & averaged here, :50-59) or already the
    clipped per-row mean [b]."""
    b = obs.shape[0]
    j = np.asarray(denoising_inds)
    if rnd is round_fp16:                    # the fp16 gradient images use the row-tied scale
        rnd = round_fp16_rows(b if denom is None else denom)
    t = ft_steps - 1 - j                                          # :456-458
    eps, acache = diffusion_mlp_forward(p_ft, chains_prev, t * _tstride(sched), obs, rnd=rnd, round_h3=round_h3)
    mu, logvar, pm = p_mean_var(sched, eps, chains_prev, t)
    std = np.clip(np.exp(0.5 * logvar), min_logprob_std, 1e6)
    lp_el = gaussian_logprob(chains_next, mu, std)
    in_clip = (lp_el >= -5) & (lp_el <= 2)
    lp_el_c = np.clip(lp_el, -5, 2)                               # :50
    H = min(reward_horizon, lp_el.shape[1])                       # :54-55
    newlp = lp_el_c[:, :H].mean(axis=(1, 2))                      # :58
    if np.ndim(oldlogprobs) == 3:
        oldlp = np.clip(oldlogprobs, -5, 2)[:, :H].mean(axis=(1, 2))
    else:
        oldlp = np.asarray(oldlogprobs, np.float64)
    adv = np.asarray(advantages, np.float64)
    if norm_adv:                                                  # :74-75 (population std)
        am, asd = (adv.mean(), adv.std()) if adv_mean_std is None else adv_mean_std
        adv = (adv - am) / (asd + 1e-8)
    D = b if denom is None else denom
    disc = gamma_denoising ** (ft_steps - j.astype(np.float64) - 1)  # :83-86
    adv = adv * disc
    logratio = newlp - oldlp                                      # :89
    ratio = np.exp(logratio)
    tf_ = j.astype(np.float64) / (ft_steps - 1) if ft_steps > 1 else j.astype(np.float64)
    if ft_steps > 1:                                              # :93-101
        cc = clip_ploss_coef_base + (clip_ploss_coef - clip_ploss_coef_base) * (
            np.exp(clip_ploss_coef_rate * tf_) - 1) / (math.exp(clip_ploss_coef_rate) - 1)
    else:
        cc = tf_
    pg1 = -adv * ratio
    rclip = np.clip(ratio, 1 - cc, 1 + cc)
    pg2 = -adv * rclip
    pg_loss = np.maximum(pg1, pg2).sum() / D                      # :104-106
    cw = None
    if critic_dedup is not None:
        # the value loss depends on the sample only: evaluate each distinct sample once with its
        # multiplicity as the weight (the same sums; with rnd, the kernels' rounding points of
        # their sample-weighted critic rows, csrc/update.hip crit_compact_kernel)
        first, mult = critic_dedup
        first = np.asarray(first)
        cw = np.asarray(mult, np.float64)
        obs, returns = obs[first], np.asarray(returns, np.float64)[first]
        if oldvalues is not None:
            oldvalues = np.asarray(oldvalues, np.float64)[first]
    v, ccache = critic_forward(pc, obs, rnd=rnd)
    v = v[:, 0]                                                   # :109
    w_rows = cw if cw is not None else np.ones_like(v)
    if clip_vloss_coef is not None:                               # :110-116
        oldvalues = np.asarray(oldvalues, np.float64)
        vl_un = (v - returns) ** 2
        v_cl = oldvalues + np.clip(v - oldvalues, -clip_vloss_coef, clip_vloss_coef)
        vl_cl = (v_cl - returns) ** 2
        v_loss = 0.5 * (w_rows * np.maximum(vl_un, vl_cl)).sum() / D
    else:
        v_loss = 0.5 * (w_rows * (v - returns) ** 2).sum() / D   # :118
    approx_kl = ((ratio - 1) - logratio).sum() / D                # :121
    clipfrac = (np.abs(ratio - 1.0) > cc).astype(np.float64).sum() / D
    metrics = dict(pg_loss=pg_loss, entropy_loss=-1.0, v_loss=v_loss, clipfrac=clipfrac,
                   approx_kl=approx_kl, ratio=ratio.sum() / D, bc_loss=0.0, eta=1.0,
                   loss=pg_loss + vf_coef * v_loss)
    if not with_grad:
        return metrics, None, None
    # ---- gradient of loss = pg_loss + vf_coef * v_loss (train_ppo_diffusion_agent.py:340) ----
    # tf.maximum routes ties to the first argument; tf.clip_by_value passes grads inside [lo, hi].
    take1 = pg1 >= pg2
    ratio_in = (ratio >= 1 - cc) & (ratio <= 1 + cc)
    dpg_dratio = np.where(take1, -adv, np.where(ratio_in, -adv, 0.0)) / D
    dnewlp = dpg_dratio * ratio
    dlp_el = np.zeros_like(lp_el)
    dlp_el[:, :H] = (dnewlp / (H * lp_el.shape[2]))[:, None, None]
    dlp_el = dlp_el * in_clip
    dmu = dlp_el * (chains_next - mu) / std ** 2
    dxr = dmu * pm["m1"] * pm["unclipped"]
    deps = -pm["c2"] * dxr
    xdim = chains_prev.shape[1] * chains_prev.shape[2]
    ga = diffusion_mlp_backward(p_ft, acache, deps, xdim)
    if clip_vloss_coef is not None:
        # tf.maximum's gradient to its first argument on ties; tf.clip_by_value's passes inside [-c, c]
        d_old = v - oldvalues
        inside = (d_old >= -clip_vloss_coef) & (d_old <= clip_vloss_coef)
        dv = vf_coef * np.where(vl_un >= vl_cl, v - returns, np.where(inside, v_cl - returns, 0.0)) / D
    else:
        dv = vf_coef * (v - returns) / D
    if cw is not None:
        dv = dv * cw
    gc, _ = residual_mlp_backward(pc, ccache, dv[:, None], "Mish", "")
    if eta_grad:
        # d loss / d eta (learnable DDIM eta, parity unpinned): mu = c2 x0 + c3 x moves through
        # d (dmu/deta = dd/deta * eps', eps' the noise recomputed from the clipped x0) and the
        # Normal's std through sigma (diffusion_vpg.py:219-234, 417-422)
        dd, dstd = ddim_eta_grad_terms(sched, t, sched["ddim_eta"], min_logprob_std)
        sh = (-1,) + (1,) * (chains_prev.ndim - 1)
        a = sched["ddim_alphas"].astype(np.float64)[t].reshape(sh)
        x0 = np.clip(pm["c1"] * chains_prev - pm["c2"] * eps, -1.0, 1.0)
        e2 = (chains_prev - np.sqrt(a) * x0) / np.sqrt(1.0 - a)
        r = chains_next - mu
        dlp_deta = r / std ** 2 * dd.reshape(sh) * e2 + (r ** 2 / std ** 3 - 1.0 / std) * dstd.reshape(sh)
        metrics["d_eta"] = float((dlp_el * dlp_deta).sum())
    return metrics, ga, gc


# ----------------------------------------------------------------------------------------------
# §8(f) row 3: pretraining loss (model/diffusion/diffusion.py:179-202, predict_epsilon = True)
# ----------------------------------------------------------------------------------------------
def q_sample(sched, x_start, t, noise):
    """diffusion.py:196-202: sqrt(ac_t) x_0 + sqrt(1 - ac_t) noise, the buffers in fp32 (:62-65)."""
    ac = np.asarray(sched["alphas_cumprod"], np.float32)
    sa = np.sqrt(ac).astype(np.float32)[t]
    s1 = np.sqrt(np.float32(1.0) - ac).astype(np.float32)[t]
    shape = (-1,) + (1,) * (np.ndim(x_start) - 1)
    return sa.reshape(shape).astype(np.float64) * x_start + s1.reshape(shape).astype(np.float64) * noise


def p_losses(p, sched, x_start, state, t, noise, with_grad=True, rnd=None, denom=None, round_h3=False):
    """diffusion.py:186-194: loss = mean((network(q_sample(x_0, t, noise), t, cond) - noise)^2) and
    its parameter gradient. x_start, noise [B,Ta,Da]; state [B,To,Do]; t [B] int (the draws of
    :182 and :187 are inputs here). denom overrides the element count of the mean (data-parallel
    shards: summing per-shard gradients with the global count gives the full-batch one)."""
    xn = q_sample(sched, x_start, np.asarray(t), noise)
    if rnd is round_fp16:                    # the fp16 gradient images use the row-tied scale
        xd = x_start.shape[1] * x_start.shape[2]
        rnd = round_fp16_rows(x_start.shape[0] if denom is None else denom // xd)
    eps, cache = diffusion_mlp_forward(p, xn, np.asarray(t), state, rnd=rnd, round_h3=round_h3)
    e = eps - noise
    n = e.size if denom is None else denom
    loss = float((e ** 2).sum() / n)
    if not with_grad:
        return loss, None
    deps = 2.0 * e / n
    return loss, diffusion_mlp_backward(p, cache, deps, x_start.shape[1] * x_start.shape[2])


# ----------------------------------------------------------------------------------------------
# a14: Keras 3 AdamW step (train_ppo_agent.py:45-49; semantics in SURVEY.md §8 quirk 2)
# ----------------------------------------------------------------------------------------------
def keras_adamw_step(param, grad, m, v, step, lr=1e-4, wd=0.004, beta1=0.9, beta2=0.999, eps=1e-7):
    """step is the 1-based iteration count. Decoupled decay first, then Adam. Returns new (p,m,v)."""
    p = np.asarray(param, np.float64)
    g = np.asarray(grad, np.float64)
    p = p - p * wd * lr
    m = m + (g - m) * (1 - beta1)
    v = v + (g * g - v) * (1 - beta2)
    alpha = lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    p = p - (m * alpha) / (np.sqrt(v) + eps)
    return p, m, v


def torch_adamw_step(param, grad, m, v, step, lr=1e-4, wd=0.0, beta1=0.9, beta2=0.999, eps=1e-8):
    """Documented alternative (PyTorch AdamW ordering/epsilon placement)."""
    p = np.asarray(param, np.float64) * (1 - lr * wd)
    m = beta1 * m + (1 - beta1) * grad
    v = beta2 * v + (1 - beta2) * grad * grad
    mh = m / (1 - beta1 ** step)
    vh = v / (1 - beta2 ** step)
    return p - lr * mh / (np.sqrt(vh) + eps), m, v


# ----------------------------------------------------------------------------------------------
# a18: RunningRewardScaler (util/reward_scaling.py:13-87)
# ----------------------------------------------------------------------------------------------
class RunningRewardScalerOracle:
    """util/reward_scaling.py:13-87. per_env=True keeps the reference's shapes: RunningMeanStd of
    shape (num_envs,) updated with rets [E, S] reduced over axis 0 (the envs, :23-27, :65), joined by
    NumPy broadcasting (so S == num_envs, or a length-1 side)."""

    def __init__(self, num_envs, cliprew=10.0, gamma=0.99, epsilon=1e-8, per_env=False):
        shape = (num_envs,) if per_env else ()
        self.mean, self.var, self.count = np.zeros(shape), np.ones(shape), 1e-4   # :19-21
        if not per_env:
            self.mean, self.var = 0.0, 1.0
        self.per_env = per_env
        self.ret = np.zeros(num_envs)
        self.cliprew, self.gamma, self.epsilon = cliprew, gamma, epsilon

    def __call__(self, reward, first):
        """reward, first: [E, S] (the agent passes reward_trajs.T, firsts[:-1].T, agent :232-236)."""
        rets = np.zeros_like(reward, dtype=np.float64)
        prev = self.ret
        for t in range(reward.shape[1]):                          # :84-87
            prev = rets[:, t] = reward[:, t] + (1 - first[:, t]) * self.gamma * prev
        self.ret = rets[:, -1]
        x = rets if self.per_env else rets.reshape(-1)            # :65
        bm, bv, bc = x.mean(axis=0), x.var(axis=0), x.shape[0]    # :23-27
        delta = bm - self.mean                                    # :29-39
        tot = self.count + bc
        self.mean = self.mean + delta * bc / tot
        M2 = self.var * self.count + bv * bc + delta ** 2 * self.count * bc / tot
        self.var = M2 / (tot - 1)
        self.count = tot
        return np.clip(reward / np.sqrt(self.var + self.epsilon), -self.cliprew, self.cliprew)


# ----------------------------------------------------------------------------------------------
# a19: GAE (train_ppo_diffusion_agent.py:239-263)
# ----------------------------------------------------------------------------------------------
def gae(rewards, values, last_values, terminated, gamma=0.99, lam=0.95, reward_scale_const=1.0):
    """rewards/values/terminated [S,E]; last_values [E] = critic(obs after last step)."""
    S = rewards.shape[0]
    adv = np.zeros_like(rewards, dtype=np.float64)
    last = 0.0
    for t in reversed(range(S)):
        nextv = last_values if t == S - 1 else values[t + 1]
        nonterm = 1.0 - terminated[t]
        delta = rewards[t] * reward_scale_const + gamma * nextv * nonterm - values[t]
        last = delta + gamma * lam * nonterm * last
        adv[t] = last
    return adv, adv + values


# ----------------------------------------------------------------------------------------------
# a20: minibatch index math (train_ppo_diffusion_agent.py:282-312)
# ----------------------------------------------------------------------------------------------
def minibatch_indices(perm, batch, batch_size, ft_steps):
    start = batch * batch_size
    inds = perm[start:start + batch_size]
    return inds // ft_steps, inds % ft_steps                       # tf.unravel_index


def num_batches(total, batch_size):
    return max(1, total // batch_size)                             # :288


# ----------------------------------------------------------------------------------------------
# a16: episode accounting (train_ppo_diffusion_agent.py:144-183)
# ----------------------------------------------------------------------------------------------
def episode_stats(firsts, rewards, act_steps, success_threshold=3.0):
    n_envs = firsts.shape[1]
    eps_ = []
    for e in range(n_envs):
        idx = np.where(firsts[:, e] == 1)[0]
        for i in range(len(idx) - 1):
            if idx[i + 1] - idx[i] > 1:
                eps_.append((e, idx[i], idx[i + 1] - 1))
    if not eps_:
        return dict(num_episode_finished=0, avg_episode_reward=0.0, avg_best_reward=0.0,
                    success_rate=0.0)
    split = [rewards[s:en + 1, e] for e, s, en in eps_]
    er = np.array([r.sum() for r in split])
    best = np.array([r.max() / act_steps for r in split])
    return dict(num_episode_finished=len(split), avg_episode_reward=float(er.mean()),
                avg_best_reward=float(best.mean()), success_rate=float((best >= success_threshold).mean()))


def explained_variance(values, returns):
    """train_ppo_diffusion_agent.py:373-377."""
    var_y = np.var(returns)
    return np.nan if var_y == 0 else 1 - np.var(returns - values) / var_y


# ----------------------------------------------------------------------------------------------
# synthetic weights (Keras glorot_uniform kernel, zero bias) — SURVEY.md §8(d)
# ----------------------------------------------------------------------------------------------
def glorot(rng, fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(np.float32)


def init_actor(rng, obs_dim=11, action_dim=3, horizon=4, cond_steps=1, time_dim=16, hidden=512,
               bias_scale=0.0):
    xdim = action_dim * horizon
    ind = xdim + time_dim + obs_dim * cond_steps
    p = {"time_w1": glorot(rng, time_dim, 2 * time_dim), "time_b1": np.zeros(2 * time_dim, np.float32),
         "time_w2": glorot(rng, 2 * time_dim, time_dim), "time_b2": np.zeros(time_dim, np.float32),
         "in_w": glorot(rng, ind, hidden), "in_b": np.zeros(hidden, np.float32),
         "l1_w": glorot(rng, hidden, hidden), "l1_b": np.zeros(hidden, np.float32),
         "l2_w": glorot(rng, hidden, hidden), "l2_b": np.zeros(hidden, np.float32),
         "out_w": glorot(rng, hidden, xdim), "out_b": np.zeros(xdim, np.float32)}
    if bias_scale:
        for k in list(p):
            if k.endswith("_b") or k.endswith("b1") or k.endswith("b2"):
                p[k] = rng.uniform(-bias_scale, bias_scale, size=p[k].shape).astype(np.float32)
    return p


def init_critic(rng, obs_dim=11, cond_steps=1, hidden=256, bias_scale=0.0):
    ind = obs_dim * cond_steps
    p = {"in_w": glorot(rng, ind, hidden), "in_b": np.zeros(hidden, np.float32),
         "l1_w": glorot(rng, hidden, hidden), "l1_b": np.zeros(hidden, np.float32),
         "l2_w": glorot(rng, hidden, hidden), "l2_b": np.zeros(hidden, np.float32),
         "out_w": glorot(rng, hidden, 1), "out_b": np.zeros(1, np.float32)}
    if bias_scale:
        for k in list(p):
            if k.endswith("_b"):
                p[k] = rng.uniform(-bias_scale, bias_scale, size=p[k].shape).astype(np.float32)
    return p

"""CPU tests of the oracle itself: pinned against the reference's own module (reward scaling
goldens), published known-answer vectors (Philox), SURVEY fp32 schedule goldens, and an
independent autograd restatement for the gradients."""
import os

import numpy as np
import pytest

from oracle import dppo_oracle as O
from oracle import philox as PX
from tests.helpers import HOPPER, make_models, to_f64

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_schedule_matches_survey_goldens():
    s = O.ddpm_schedule(20)
    std = np.exp(0.5 * s["ddpm_logvar_clipped"].astype(np.float64))
    assert abs(s["betas"][0] - 0.007993) < 1e-6 and s["betas"][19] == np.float32(0.999)
    assert abs(s["alphas_cumprod"][19] - 6.0596e-6) < 1e-9
    np.testing.assert_allclose(std[[0, 1, 9, 19]], [1e-10, 0.07583, 0.33921, 0.99647], rtol=2e-4)
    assert abs(s["ddpm_mu_coef1"][0] - 0.999997) < 1e-6 and s["ddpm_mu_coef2"][0] == 0
    assert abs(s["sqrt_recip_alphas_cumprod"][19] - 406.237) < 1e-3


def test_product_schedule_equals_oracle():
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddpm_buffers
    a, b = O.ddpm_schedule(20), ddpm_buffers(20)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_reward_scaler_matches_reference_goldens():
    g = np.load(os.path.join(GOLD, "reward_scaling.npz"))
    ci = 0
    while f"c{ci}_meta" in g:
        E, S, n_calls = g[f"c{ci}_meta"]
        orc = O.RunningRewardScalerOracle(int(E))
        for k in range(int(n_calls)):
            p = f"c{ci}_k{k}_"
            out = orc(g[p + "reward"], g[p + "first"])
            np.testing.assert_allclose(out, g[p + "out"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose([orc.mean, orc.var, orc.count], g[p + "rms"], rtol=1e-12)
            np.testing.assert_allclose(orc.ret, g[p + "ret"], rtol=1e-12)
        ci += 1
    assert ci == 4


def test_reward_scaler_per_env_matches_reference_goldens():
    """per_env=True (reward_scaling.py:51-66): the restatement against the reference's own outputs
    (tests/golden/reward_scaling_per_env.npz), broadcasting cases and the rejected shape included."""
    g = np.load(os.path.join(GOLD, "reward_scaling_per_env.npz"))
    ci = 0
    while f"c{ci}_meta" in g:
        E, n_calls = (int(x) for x in g[f"c{ci}_meta"])
        orc = O.RunningRewardScalerOracle(E, per_env=True)
        for k in range(n_calls):
            p = f"c{ci}_k{k}_"
            if p + "raises" in g:
                with pytest.raises(ValueError):
                    orc(g[p + "reward"], g[p + "first"])
                break
            out = orc(g[p + "reward"], g[p + "first"])
            assert out.shape == g[p + "out"].shape
            np.testing.assert_allclose(out, g[p + "out"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(orc.mean, g[p + "mean"], rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(orc.var, g[p + "var"], rtol=1e-12)
            np.testing.assert_allclose(orc.count, g[p + "count"], rtol=1e-12)
            np.testing.assert_allclose(orc.ret, g[p + "ret"], rtol=1e-12)
        ci += 1
    assert ci == 6


def test_philox_known_answers():
    """Random123 kat_vectors for philox4x32_10."""
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for c, k, want in kat:
        assert tuple(int(x) for x in PX.philox4x32_10(*c, *k)) == want


def test_normals_are_standard():
    z = PX.sampler_normals(7, 3, 0, 4096, 12, 5).ravel()
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02


@pytest.mark.parametrize("n", [1, 2, 5, 13, 1000, 4097, 320000])
def test_feistel_is_bijection(n):
    p = PX.feistel_permute(np.arange(n), n, 42, 3)
    assert np.array_equal(np.sort(p), np.arange(n))


def test_gae_against_direct_loop():
    rng = np.random.default_rng(0)
    S, E = 30, 5
    r, v, lv = rng.normal(size=(S, E)), rng.normal(size=(S, E)), rng.normal(size=E)
    term = (rng.uniform(size=(S, E)) < 0.1).astype(float)
    a, ret = O.gae(r, v, lv, term)
    for e in range(E):
        last = 0.0
        for t in reversed(range(S)):
            nv = lv[e] if t == S - 1 else v[t + 1, e]
            d = r[t, e] + 0.99 * nv * (1 - term[t, e]) - v[t, e]
            last = d + 0.99 * 0.95 * (1 - term[t, e]) * last
            assert abs(a[t, e] - last) < 1e-12
    np.testing.assert_allclose(ret, a + v)


def _torch_closs(base, ft, critic, sched, obs, prev, nxt, j, ret, adv, oldlp, kf, oldv=None, clip_v=None):
    """Independent restatement with torch float64 autograd (checker for the oracle's backward)."""
    import torch
    T = lambda x: torch.tensor(np.asarray(x, np.float64))
    P = {k: T(v).requires_grad_(True) for k, v in ft.items()}
    C = {k: T(v).requires_grad_(True) for k, v in critic.items()}
    mish = lambda x: x * torch.tanh(torch.nn.functional.softplus(x))
    b = obs.shape[0]
    t = kf - 1 - j
    half = 8
    freqs = torch.exp(torch.arange(half, dtype=torch.float64) * -(np.log(10000) / (half - 1)))
    e = T(t)[:, None] * freqs[None]
    e = torch.cat([torch.sin(e), torch.cos(e)], -1)
    temb = mish(e @ P["time_w1"] + P["time_b1"]) @ P["time_w2"] + P["time_b2"]
    x = T(prev).reshape(b, -1)
    inp = torch.cat([x, temb, T(obs).reshape(b, -1)], -1)
    h1 = inp @ P["in_w"] + P["in_b"]
    h2 = torch.relu(h1) @ P["l1_w"] + P["l1_b"]
    h3 = torch.relu(h2) @ P["l2_w"] + P["l2_b"] + h1
    eps = h3 @ P["out_w"] + P["out_b"]
    c1 = T(sched["sqrt_recip_alphas_cumprod"].astype(np.float64)[t])[:, None]
    c2 = T(sched["sqrt_recipm1_alphas_cumprod"].astype(np.float64)[t])[:, None]
    m1 = T(sched["ddpm_mu_coef1"].astype(np.float64)[t])[:, None]
    m2 = T(sched["ddpm_mu_coef2"].astype(np.float64)[t])[:, None]
    lv = T(sched["ddpm_logvar_clipped"].astype(np.float64)[t])[:, None]
    xr = torch.clamp(c1 * x - c2 * eps, -1, 1)
    mu = m1 * xr + m2 * x
    std = torch.clamp(torch.exp(0.5 * lv), 0.1, 1e6)
    lp = torch.distributions.Normal(mu, std).log_prob(T(nxt).reshape(b, -1))
    newlp = torch.clamp(lp, -5, 2).mean(-1)
    A = T(adv)
    A = (A - A.mean()) / (A.std(unbiased=False) + 1e-8)
    A = A * 0.99 ** (kf - T(j) - 1)
    ratio = torch.exp(newlp - T(oldlp))
    pg = torch.max(-A * ratio, -A * torch.clamp(ratio, 0.99, 1.01)).mean()
    h1 = T(obs).reshape(b, -1) @ C["in_w"] + C["in_b"]
    h2 = mish(h1) @ C["l1_w"] + C["l1_b"]
    h3 = mish(h2) @ C["l2_w"] + C["l2_b"] + h1
    V = (h3 @ C["out_w"] + C["out_b"])[:, 0]
    if clip_v is None:
        vl = 0.5 * ((V - T(ret)) ** 2).mean()
    else:   # diffusion_ppo.py:110-116
        vc = T(oldv) + torch.clamp(V - T(oldv), -clip_v, clip_v)
        vl = 0.5 * torch.maximum((V - T(ret)) ** 2, (vc - T(ret)) ** 2).mean()
    (pg + 0.5 * vl).backward()
    return ({k: v.grad.numpy() for k, v in P.items()}, {k: v.grad.numpy() for k, v in C.items()},
            float(pg), float(vl))


def test_oracle_closs_gradient_matches_autograd():
    base, ft, critic = make_models(0, HOPPER)
    sched = O.ddpm_schedule(20)
    rng = np.random.default_rng(1)
    b, kf = 64, 10
    obs = rng.uniform(-1, 1, (b, 1, 11))
    prev = rng.normal(0, 0.5, (b, 4, 3))
    nxt = prev + rng.normal(0, 0.1, (b, 4, 3))
    j = rng.integers(0, kf, b)
    ret, adv = rng.normal(size=b), rng.normal(size=b)
    oldlp = rng.normal(0.5, 0.3, b)
    m, ga, gc = O.c_loss(to_f64(ft), to_f64(critic), sched, obs, prev, nxt, j, ret, None, adv, oldlp, kf)
    ta, tc, pg, vl = _torch_closs(base, ft, critic, sched, obs, prev, nxt, j, ret, adv, oldlp, kf)
    assert abs(m["pg_loss"] - pg) < 1e-12 and abs(m["v_loss"] - vl) < 1e-12
    for k in ta:
        np.testing.assert_allclose(ga[k], ta[k], rtol=1e-8, atol=1e-12, err_msg=k)
    for k in tc:
        np.testing.assert_allclose(gc[k], tc[k], rtol=1e-8, atol=1e-12, err_msg=k)


def test_oracle_clipped_value_loss_gradient_matches_autograd():
    """clip_vloss_coef (diffusion_ppo.py:110-116): the oracle's v_loss and critic gradient against torch
    float64 autograd, old values V(obs) + U(-0.4, 0.4) at c = 0.2 (both branches of the max, both sides
    of the clip), with and without the sample-dedup weighting the kernels use (repeated samples)."""
    base, ft, critic = make_models(0, HOPPER)
    sched = O.ddpm_schedule(20)
    rng = np.random.default_rng(2)
    b, kf = 64, 10
    obs = rng.uniform(-1, 1, (b, 1, 11))
    obs[32:] = obs[:32]                                    # every sample twice (dedup weights 2)
    prev = rng.normal(0, 0.5, (b, 4, 3))
    nxt = prev + rng.normal(0, 0.1, (b, 4, 3))
    j = rng.integers(0, kf, b)
    ret, adv = rng.normal(size=b), rng.normal(size=b)
    ret[32:] = ret[:32]
    oldlp = rng.normal(0.5, 0.3, b)
    v_now = O.critic_forward(to_f64(critic), obs)[0][:, 0]
    oldv = v_now + rng.uniform(-0.4, 0.4, b)
    oldv[32:] = oldv[:32]
    ta, tc, pg, vl = _torch_closs(base, ft, critic, sched, obs, prev, nxt, j, ret, adv, oldlp, kf, oldv, 0.2)
    d = np.abs(v_now - oldv)
    assert (d > 0.2).any() and (d < 0.2).any()
    for dedup in (None, (np.arange(32), np.full(32, 2))):
        m, ga, gc = O.c_loss(to_f64(ft), to_f64(critic), sched, obs, prev, nxt, j, ret, oldv, adv, oldlp, kf,
                             clip_vloss_coef=0.2, critic_dedup=dedup)
        assert abs(m["v_loss"] - vl) < 1e-12
        for k in tc:
            np.testing.assert_allclose(gc[k], tc[k], rtol=1e-8, atol=1e-12, err_msg=k)


def test_keras_adamw_first_step():
    p, g = np.array([1.0, -2.0]), np.array([0.5, -0.25])
    newp, m, v = O.keras_adamw_step(p, g, np.zeros(2), np.zeros(2), 1, lr=1e-3, wd=0.004)
    # step 1: m = 0.1 g, v = 0.001 g^2, alpha = lr sqrt(0.001)/0.1 -> update ~= lr * sign(g)
    expect = p * (1 - 0.004 * 1e-3) - 1e-3 * np.sqrt(1e-3) / 0.1 * (0.1 * g) / (np.sqrt(1e-3) * np.abs(g) + 1e-7)
    np.testing.assert_allclose(newp, expect, rtol=1e-12)


def test_episode_stats():
    firsts = np.zeros((11, 2))
    firsts[0] = 1
    firsts[4, 0] = 1
    firsts[9, 0] = 1
    rew = np.arange(20, dtype=float).reshape(10, 2)
    s = O.episode_stats(firsts, rew, 4)
    # env0 episodes: steps 0..3 and 4..8 ; env1: none complete
    assert s["num_episode_finished"] == 2
    assert abs(s["avg_episode_reward"] - (rew[0:4, 0].sum() + rew[4:9, 0].sum()) / 2) < 1e-12


def test_ddim_affine_form_matches_documented_formulas():
    """The DDIM schedule rows the kernels run (affine: x0 = c0 x - c1 eps, clip, mu = c2 x0 + c3 x)
    equal the documented DDIM mean computed term by term (x0 -> clip -> eps' -> sqrt(a_prev) x0 +
    d eps', diffusion_vpg.py:193-232), on clipped and unclipped x0, for eta in {0, 0.5, 1}."""
    rng = np.random.default_rng(5)
    for eta in (0.0, 0.5, 1.0):
        sc = O.ddim_schedule(20, 10, eta)
        for j in range(10):
            x = rng.normal(0, 1.5, (64, 4, 3))
            eps = rng.normal(0, 1.5, (64, 4, 3))
            jj = np.full(64, j)
            mu_a, lv_a, _ = O.p_mean_var(sc, eps, x, jj)
            mu_d, lv_d = O.p_mean_var_ddim_direct(sc, eps, x, jj)
            np.testing.assert_allclose(mu_a, mu_d, rtol=2e-5, atol=2e-5)
            np.testing.assert_allclose(lv_a, lv_d, rtol=1e-6, atol=1e-6)


def test_ddim_host_buffers_match_oracle():
    """The product's fp32 DDIM table (model/diffusion/sampling.py, ops.sched_table) equals the
    oracle's restatement, including the eval noise rule columns."""
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddim_buffers
    for eta in (0.0, 1.0):
        tab = ops.sched_table(ddim_buffers(20, 10, eta))
        sc = O.ddim_schedule(20, 10, eta)
        for c, k in enumerate(("sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "ddpm_mu_coef1",
                               "ddpm_mu_coef2", "ddpm_logvar_clipped")):
            np.testing.assert_array_equal(tab[:, c], sc[k])
        assert (tab[:, 5] == 0).all() and (tab[:, 6] == 1).all()
        assert ddim_buffers(20, 10, eta)["time_stride"] == 2
    # DDPM rows keep the reference's eval rule: t = 0 without noise, 1e-3 floor elsewhere
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddpm_buffers
    tab = ops.sched_table(ddpm_buffers(20))
    assert tab[0, 6] == 1 and (tab[1:, 6] == 0).all() and np.allclose(tab[:, 5], 1e-3)


def test_oracle_pretrain_loss_gradient_matches_autograd():
    """p_losses (diffusion.py:186-194) in the oracle vs an independent torch float64 autograd of the
    same loss: q_sample with the fp32 buffers, DiffusionMLP, mean((eps - noise)^2)."""
    import torch
    _, ft, _ = make_models(0, HOPPER)
    sched = O.ddpm_schedule(20)
    rng = np.random.default_rng(3)
    b = 48
    x0 = rng.uniform(-1, 1, (b, 4, 3))
    obs = rng.uniform(-1, 1, (b, 1, 11))
    t = rng.integers(0, 20, b)
    noise = rng.standard_normal((b, 4, 3))
    loss, g = O.p_losses(to_f64(ft), sched, x0, obs, t, noise)
    T = lambda x: torch.tensor(np.asarray(x, np.float64))
    P = {k: T(v).requires_grad_(True) for k, v in ft.items()}
    mish = lambda x: x * torch.tanh(torch.nn.functional.softplus(x))
    half = 8
    freqs = torch.exp(torch.arange(half, dtype=torch.float64) * -(np.log(10000) / (half - 1)))
    e = T(t)[:, None] * freqs[None]
    e = torch.cat([torch.sin(e), torch.cos(e)], -1)
    temb = mish(e @ P["time_w1"] + P["time_b1"]) @ P["time_w2"] + P["time_b2"]
    ac = sched["alphas_cumprod"].astype(np.float32)
    sa = T(np.sqrt(ac).astype(np.float32)[t])[:, None]
    s1 = T(np.sqrt(np.float32(1) - ac).astype(np.float32)[t])[:, None]
    xn = sa * T(x0).reshape(b, -1) + s1 * T(noise).reshape(b, -1)
    inp = torch.cat([xn, temb, T(obs).reshape(b, -1)], -1)
    h1 = inp @ P["in_w"] + P["in_b"]
    h2 = torch.relu(h1) @ P["l1_w"] + P["l1_b"]
    h3 = torch.relu(h2) @ P["l2_w"] + P["l2_b"] + h1
    eps = h3 @ P["out_w"] + P["out_b"]
    L = ((eps - T(noise).reshape(b, -1)) ** 2).mean()
    L.backward()
    assert abs(loss - float(L)) < 1e-12
    for k, v in P.items():
        np.testing.assert_allclose(g[k], v.grad.numpy(), rtol=1e-8, atol=1e-12, err_msg=k)


def test_oracle_eta_gradient_matches_finite_differences():
    """d loss / d eta of the learnable DDIM eta (oracle c_loss eta_grad, parity unpinned: the
    reference's eta module is absent) against central differences of the oracle's own pg_loss with
    the DDIM schedule rebuilt in float64 at eta +- h, for etas whose rows hit both the std clip
    (sigma < min_logprob_std) and the free branch."""
    base, ft, critic = make_models(0, HOPPER)
    rng = np.random.default_rng(7)
    b, kf = 48, 10
    obs = rng.uniform(-1, 1, (b, 1, 11))
    prev = rng.normal(0, 0.5, (b, 4, 3))
    nxt = prev + rng.normal(0, 0.2, (b, 4, 3))
    j = rng.integers(0, kf, b)
    ret, adv = rng.normal(size=b), rng.normal(size=b)
    oldlp = rng.normal(0.0, 0.2, b)
    for eta in (0.3, 0.7, 1.0):
        sc = O.ddim_schedule(20, 10, eta, dtype=np.float64)
        args = (to_f64(ft), to_f64(critic))
        rest = (obs, prev, nxt, j, ret, None, adv, oldlp, kf)
        m, _, _ = O.c_loss(*args, sc, *rest, eta_grad=True)
        h = 1e-6
        lp = O.c_loss(*args, O.ddim_schedule(20, 10, eta + h, dtype=np.float64), *rest, with_grad=False)[0]["pg_loss"]
        lm = O.c_loss(*args, O.ddim_schedule(20, 10, eta - h, dtype=np.float64), *rest, with_grad=False)[0]["pg_loss"]
        fd = (lp - lm) / (2 * h)
        assert abs(m["d_eta"]) > 1e-4
        assert abs(m["d_eta"] - fd) <= 1e-6 * max(1.0, abs(fd)), (eta, m["d_eta"], fd)
    # the EtaFixed parametrisation round-trips
    lg = O.eta_logit_init(0.5, 0.1, 1.0)
    assert abs(O.eta_from_logit(lg, 0.1, 1.0) - 0.5) < 1e-12


def test_bc_loss_samples_every_step_with_the_base_policy():
    """c_loss's behaviour-cloning term (diffusion_ppo.py:63-71): `call(..., use_base_policy=True)` runs
    every denoising step, the fine-tuned steps included, on the frozen base actor (diffusion_vpg.py:175-176),
    and the log-probs of those chains are taken under actor_ft (use_base_policy=False), clipped to [-5, 2]."""
    base, ft, _ = make_models(seed=4)
    base, ft = to_f64(base), to_f64(ft)
    K, kf, E = 20, 10, 6
    rng = np.random.default_rng(2)
    st = rng.uniform(-1, 1, (E, 1, 11))
    xT, z = rng.standard_normal((E, 4, 3)), rng.standard_normal((K, E, 4, 3))
    sched = O.ddpm_schedule(K)
    v = O.bc_loss(base, ft, sched, st, xT, z, kf)
    _, ch = O.sample(base, base, sched, st, xT, z, kf, round_h3=False)
    assert v == -np.clip(O.get_logprobs(ft, sched, st, ch, kf), -5, 2).mean()
    _, ch_mix = O.sample(base, ft, sched, st, xT, z, kf, round_h3=False)   # the rollout's actor mix
    assert not np.allclose(ch, ch_mix)

"""GPU parity: every HIP entry point vs the float64 oracle on the same seeded inputs.

Tolerances: fp32 (f32-input MFMA) mode is checked tightly; bf16 mode (bf16 operands, fp32
accumulate/epilogue) against a stated looser bound. Integer work (Feistel permutation) is bit-exact.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import dppo_oracle as O
from oracle import philox as PX
from tests.helpers import HOPPER, HOPPER_DDIM, NARROW, WALKER, make_models, to_f64

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(dims, cuda, seed=0, eta=1.0):
    """dims with time_stride > 1 are DDIM: sched is then the oracle's DDIM restatement and tab the
    product's table (model/diffusion/sampling.py ddim_buffers) for the same (K, S, eta)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddim_buffers, ddpm_buffers
    d = ops.ModelDims(**dims)
    base, ft, critic = make_models(seed, {k: v for k, v in dims.items() if k != "time_stride"})
    if d.time_stride > 1:
        K = d.denoising_steps * d.time_stride
        sched = O.ddim_schedule(K, d.denoising_steps, eta)
        tab = torch.tensor(ops.sched_table(ddim_buffers(K, d.denoising_steps, eta)), device=cuda)
    else:
        sched = ddpm_buffers(d.denoising_steps)
        tab = torch.tensor(ops.sched_table(sched), device=cuda)
    fa = lambda p: torch.tensor(ops.flatten_params(ops.actor_param_spec(d), p), device=cuda)
    fc = lambda p: torch.tensor(ops.flatten_params(ops.critic_param_spec(d), p), device=cuda)
    return d, base, ft, critic, sched, tab, fa(base), fa(ft), fc(critic)


def _rnd(precision):
    return {"bf16": O.round_bf16, "fp16": O.round_fp16}.get(precision)


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 2e-3), ("fp16", 1e-3)])
@pytest.mark.parametrize("dims", [HOPPER, WALKER], ids=["hopper", "walker"])
def test_sampler_injected_noise(cuda, precision, tol, dims):
    """fp32: vs the exact f64 oracle. bf16: vs the oracle rounding operands to bf16 at the
    kernel's rounding points (fp32 accumulation order and rare rounding-boundary flips remain)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    E = 37  # ragged: not a multiple of the 16-row tile
    rng = np.random.default_rng(1)
    state = rng.uniform(-1, 1, (E, d.cond_steps, d.obs_dim)).astype(np.float32)
    xT = rng.standard_normal((E, d.horizon_steps, d.action_dim)).astype(np.float32)
    z = rng.standard_normal((d.denoising_steps, E, d.horizon_steps, d.action_dim)).astype(np.float32)
    split = ops.sampler_layout(d, precision, E) > 0
    # bf16 / fp16 at 37 envs run the split sampler by default; fp32 too at hopper's width (r06: the folded
    # kernel at P = 8 members of 4 waves, fp32 operands), walker2d's fp32 streams the weights
    assert split == (precision != "fp32" or d.xd == 12), (precision, d.xd)
    if split and precision == "fp32":
        assert ops.sampler_plan(d, precision, E)["members"] == 8
    ref_a, ref_c = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps,
                            rnd=_rnd(precision), round_h3=not split)
    packb, packf = ops.pack_actor(d, pb, precision), ops.pack_actor(d, pf, precision)
    act, ch = ops.sample(d, precision, packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                         x_T=torch.tensor(xT.reshape(E, -1), device=cuda),
                         noise=torch.tensor(z.reshape(d.denoising_steps, E, -1), device=cuda))
    torch.cuda.synchronize()
    act = act.cpu().numpy().reshape(ref_a.shape)
    ch = ch.cpu().numpy().reshape(ref_c.shape)
    err_a = np.abs(act - ref_a).max()
    err_c = np.abs(ch - ref_c).max()
    if precision == "fp32":
        assert err_a < tol and err_c < tol, (err_a, err_c)
    else:
        # the t=19 x0 reconstruction amplifies eps differences by 406 before its clip, so a rare
        # bf16 rounding-boundary flip can move one element; bound the 99th percentile tightly
        q99 = np.quantile(np.abs(act - ref_a), 0.99)
        assert q99 < tol and np.abs(ch - ref_c).mean() < tol, (q99, err_a, err_c)


def test_sampler_philox_stream(cuda):
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    E, seed, call = 19, 1234567890123, 7
    rng = np.random.default_rng(2)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    xT = PX.sampler_normals(seed, call, 0, E, d.xd, d.denoising_steps).reshape(E, d.horizon_steps, d.action_dim)
    z = np.stack([PX.sampler_normals(seed, call, 0, E, d.xd, i) for i in range(d.denoising_steps)])
    z = z.reshape(d.denoising_steps, E, d.horizon_steps, d.action_dim)
    ref_a, ref_c = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps)
    packb, packf = ops.pack_actor(d, pb, "fp32"), ops.pack_actor(d, pf, "fp32")
    act, ch = ops.sample(d, "fp32", packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                         seed=seed, call_id=call)
    torch.cuda.synchronize()
    assert np.abs(act.cpu().numpy().reshape(ref_a.shape) - ref_a).max() < 1e-3


@pytest.mark.parametrize("E,dims", [(1, HOPPER), (16, HOPPER), (64, HOPPER), (130, HOPPER), (256, WALKER),
                                    (512, HOPPER), (513, HOPPER)],
                         ids=["1", "16", "64-config2", "130", "256-walker-config3", "512", "513"])
def test_sampler_bf16_sizes_philox(cuda, E, dims):
    """bf16 sampler with its own Philox noise at group boundaries (1, 16), the BASELINE config-2
    shape (hopper, 64 envs), a ragged multi-XCD size (130 envs = 9 groups), config 3's shape
    (walker2d, XD = 24, 256 envs), the split kernel's maximum (512 envs = 256 workgroups) and one
    env past it (513: the weight-streaming kernel). Checked against the oracle rounding at the
    kernel's rounding points, given the same Philox draws: 99th percentile and mean tight; the
    maximum bounded loosely (the t=19 x0 reconstruction multiplies eps by 406 before its clip, so a
    single bf16 rounding-boundary flip can move one element)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    split = ops.sampler_layout(d, "bf16", E) > 0
    assert split == (E <= 512)
    if split:   # every split shape runs the folded 2-member kernel (walker2d's since r06: its TIN ring)
        assert ops.sampler_plan(d, "bf16", E)["kernel"] == 2, ops.sampler_plan(d, "bf16", E)
    seed, call = 987654321, 3
    rng = np.random.default_rng(E)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    xT = PX.sampler_normals(seed, call, 0, E, d.xd, d.denoising_steps).reshape(E, d.horizon_steps, d.action_dim)
    z = np.stack([PX.sampler_normals(seed, call, 0, E, d.xd, i) for i in range(d.denoising_steps)])
    z = z.reshape(d.denoising_steps, E, d.horizon_steps, d.action_dim)
    ref_a, ref_c = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps,
                            rnd=O.round_bf16, round_h3=not split)
    packb, packf = ops.pack_actor(d, pb, "bf16"), ops.pack_actor(d, pf, "bf16")
    act, ch = ops.sample(d, "bf16", packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                         seed=seed, call_id=call)
    torch.cuda.synchronize()
    act = act.cpu().numpy().reshape(ref_a.shape)
    ch = ch.cpu().numpy().reshape(ref_c.shape)
    assert np.isfinite(act).all() and np.isfinite(ch).all()
    dev = np.abs(act - ref_a)
    assert np.quantile(dev, 0.99) < 2e-3 and np.abs(ch - ref_c).mean() < 2e-3, (dev.max(), np.quantile(dev, 0.99))
    assert dev.max() < 0.1, dev.max()


def test_sampler_fp16_ddim_config5(cuda):
    """BASELINE config 5's per-GPU workload: DDIM 10 rows over K = 20, 512 envs per GPU, fp16
    operands, the split sampler at its maximum (256 workgroups), the kernel's own Philox noise;
    against the oracle rounding operands to fp16 at the kernel's rounding points (parity-unpinned
    like every DDIM result: the reference DDIM path cannot run)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER_DDIM, cuda)
    E, seed, call = 512, 424242, 9
    assert ops.sampler_layout(d, "fp16", E) > 0
    rng = np.random.default_rng(55)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    S = d.denoising_steps
    xT = PX.sampler_normals(seed, call, 0, E, d.xd, S).reshape(E, d.horizon_steps, d.action_dim)
    z = np.stack([PX.sampler_normals(seed, call, 0, E, d.xd, i) for i in range(S)])
    z = z.reshape(S, E, d.horizon_steps, d.action_dim)
    ref_a, ref_c = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps,
                            rnd=O.round_fp16, round_h3=False)
    packb, packf = ops.pack_actor(d, pb, "fp16"), ops.pack_actor(d, pf, "fp16")
    act, ch = ops.sample(d, "fp16", packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                         seed=seed, call_id=call)
    torch.cuda.synchronize()
    dev = np.abs(act.cpu().numpy().reshape(ref_a.shape) - ref_a)
    assert np.isfinite(dev).all()
    assert np.quantile(dev, 0.99) < 1e-3 and np.abs(ch.cpu().numpy().reshape(ref_c.shape) - ref_c).mean() < 1e-3, \
        (dev.max(), np.quantile(dev, 0.99))
    assert dev.max() < 0.1, dev.max()


def test_sampler_split_repeatable(cuda):
    """Back-to-back launches of the split sampler on the same stream reuse one exchange buffer with
    new tags: identical inputs give bit-identical outputs, launch after launch."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    E = 64
    assert ops.sampler_layout(d, "bf16", E) > 0
    rng = np.random.default_rng(9)
    cond = torch.tensor(rng.uniform(-1, 1, (E, d.sd)).astype(np.float32), device=cuda)
    packb, packf = ops.pack_actor(d, pb, "bf16"), ops.pack_actor(d, pf, "bf16")
    outs = [ops.sample(d, "bf16", packb, packf, tab, cond, seed=5, call_id=11)[0].clone() for _ in range(20)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 3e-3), ("fp16", 2e-3)])
def test_sampler_ddim(cuda, precision, tol):
    """BASELINE config 5's DDIM sampler (10 rows over K = 20, eta = 1) vs the oracle's DDIM
    restatement (parity-unpinned: the reference DDIM path cannot run)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER_DDIM, cuda)
    E, S = 37, d.denoising_steps
    rng = np.random.default_rng(21)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    xT = rng.standard_normal((E, 4, 3)).astype(np.float32)
    z = rng.standard_normal((S, E, 4, 3)).astype(np.float32)
    split = ops.sampler_layout(d, precision, E) > 0
    ref_a, ref_c = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps,
                            rnd=_rnd(precision), round_h3=not split)
    packb, packf = ops.pack_actor(d, pb, precision), ops.pack_actor(d, pf, precision)
    act, ch = ops.sample(d, precision, packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                         x_T=torch.tensor(xT.reshape(E, -1), device=cuda),
                         noise=torch.tensor(z.reshape(S, E, -1), device=cuda))
    torch.cuda.synchronize()
    act = act.cpu().numpy().reshape(ref_a.shape)
    ch = ch.cpu().numpy().reshape(ref_c.shape)
    assert ch.shape[1] == d.ft_denoising_steps + 1
    if precision == "fp32":
        assert np.abs(act - ref_a).max() < tol and np.abs(ch - ref_c).max() < tol
    else:
        assert np.quantile(np.abs(act - ref_a), 0.99) < tol and np.abs(ch - ref_c).mean() < tol


def test_sampler_ddim_eval(cuda):
    """Deterministic DDIM sampling: the eta = 0 table and no noise on any row (diffusion_vpg.py:222-224,
    303-306), fp32 vs the oracle."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER_DDIM, cuda, eta=0.0)
    E, S = 16, d.denoising_steps
    rng = np.random.default_rng(22)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    xT = rng.standard_normal((E, 4, 3)).astype(np.float32)
    z = rng.standard_normal((S, E, 4, 3)).astype(np.float32)
    ref_a, _ = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, d.ft_denoising_steps,
                        deterministic=True)
    packb, packf = ops.pack_actor(d, pb, "fp32"), ops.pack_actor(d, pf, "fp32")
    act, _ = ops.sample(d, "fp32", packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                        x_T=torch.tensor(xT.reshape(E, -1), device=cuda),
                        noise=torch.tensor(z.reshape(S, E, -1), device=cuda), deterministic=True)
    torch.cuda.synchronize()
    assert np.abs(act.cpu().numpy().reshape(ref_a.shape) - ref_a).max() < 2e-4


def test_logprob_ddim(cuda):
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER_DDIM, cuda)
    n, kf = 29, d.ft_denoising_steps
    rng = np.random.default_rng(23)
    state = rng.uniform(-1, 1, (n, 1, d.obs_dim)).astype(np.float32)
    chains = (rng.standard_normal((n, kf + 1, 4, 3)) * 0.5).astype(np.float32)
    ref = O.get_logprobs(to_f64(ft), sched, state.astype(np.float64), chains.astype(np.float64), kf)
    lpe, _ = ops.logprob(d, "fp32", ops.pack_actor(d, pf, "fp32"), tab, torch.tensor(state.reshape(n, -1), device=cuda),
                         torch.tensor(chains.reshape(n, kf + 1, -1), device=cuda))
    torch.cuda.synchronize()
    rel = np.abs(lpe.cpu().numpy().reshape(ref.shape) - ref) / (1 + np.abs(ref))
    assert rel.max() < 1e-3, rel.max()


def test_sampler_deterministic_and_empty(cuda):
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    E = 16
    rng = np.random.default_rng(3)
    state = rng.uniform(-1, 1, (E, 1, d.obs_dim)).astype(np.float32)
    xT = rng.standard_normal((E, 4, 3)).astype(np.float32)
    z = rng.standard_normal((20, E, 4, 3)).astype(np.float32)
    ref_a, _ = O.sample(to_f64(base), to_f64(ft), sched, state.astype(np.float64), xT, z, 10, deterministic=True)
    packb, packf = ops.pack_actor(d, pb, "fp32"), ops.pack_actor(d, pf, "fp32")
    act, _ = ops.sample(d, "fp32", packb, packf, tab, torch.tensor(state.reshape(E, -1), device=cuda),
                        x_T=torch.tensor(xT.reshape(E, -1), device=cuda),
                        noise=torch.tensor(z.reshape(20, E, -1), device=cuda), deterministic=True)
    torch.cuda.synchronize()
    assert np.abs(act.cpu().numpy().reshape(ref_a.shape) - ref_a).max() < 2e-4
    # E = 0 is a no-op
    ops.sample(d, "fp32", packb, packf, tab, torch.zeros(0, d.sd, device=cuda))


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 2e-3), ("fp16", 2e-3)])
@pytest.mark.parametrize("dims", [HOPPER, WALKER], ids=["hopper", "walker"])
def test_logprob(cuda, precision, tol, dims):
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    n = 45
    rng = np.random.default_rng(4)
    state = rng.uniform(-1, 1, (n, 1, d.obs_dim)).astype(np.float32)
    chains = (rng.standard_normal((n, d.ft_denoising_steps + 1, d.horizon_steps, d.action_dim)) * 0.5).astype(np.float32)
    ref = O.get_logprobs(to_f64(ft), sched, state.astype(np.float64), chains.astype(np.float64), d.ft_denoising_steps,
                         rnd=_rnd(precision))
    packf = ops.pack_actor(d, pf, precision)
    lpe, lpm = ops.logprob(d, precision, packf, tab, torch.tensor(state.reshape(n, -1), device=cuda),
                           torch.tensor(chains.reshape(n, d.ft_denoising_steps + 1, -1), device=cuda))
    torch.cuda.synchronize()
    lpe = lpe.cpu().numpy().reshape(ref.shape)
    ref_mean = np.clip(ref, -5, 2).mean(axis=(1, 2)).reshape(n, d.ft_denoising_steps)
    rel = np.abs(lpe - ref) / (1 + np.abs(ref))
    assert np.quantile(rel, 0.99) < tol, np.quantile(rel, 0.99)
    assert np.abs(lpm.cpu().numpy() - ref_mean).max() < tol * 10


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 1e-3), ("fp16", 1e-3)])
def test_critic_forward(cuda, precision, tol):
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    n = 77
    state = np.random.default_rng(5).uniform(-1, 1, (n, 1, d.obs_dim)).astype(np.float32)
    ref, _ = O.critic_forward(to_f64(critic), state.astype(np.float64), rnd=_rnd(precision))
    v = ops.critic_forward(d, precision, ops.pack_critic(d, pc, precision),
                           torch.tensor(state.reshape(n, -1), device=cuda))
    torch.cuda.synchronize()
    assert np.abs(v.cpu().numpy() - ref[:, 0]).max() < tol * (1 + np.abs(ref).max())


@pytest.mark.parametrize("S,E", [(50, 4), (500, 64), (7, 3), (1, 5)])
def test_gae(cuda, S, E):
    import torch
    from diffusionpolicyoptimization_amd import ops
    rng = np.random.default_rng(S * 100 + E)
    r = rng.normal(size=(S, E))
    v = rng.normal(size=(S, E)).astype(np.float32)
    lv = rng.normal(size=E).astype(np.float32)
    term = (rng.uniform(size=(S, E)) < 0.05).astype(np.uint8)
    ref_a, ref_r = O.gae(r, v.astype(np.float64), lv.astype(np.float64), term.astype(np.float64))
    a, ret = ops.gae(torch.tensor(r, device=cuda), torch.tensor(v, device=cuda), torch.tensor(lv, device=cuda),
                     torch.tensor(term, device=cuda))
    torch.cuda.synchronize()
    np.testing.assert_allclose(a.cpu().numpy(), ref_a, rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(ret.cpu().numpy(), ref_r, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("S,E,p", [(50, 4, 0.1), (500, 64, 0.004), (500, 512, 0.02), (7, 3, 0.0), (1, 5, 0.5)])
def test_episode_sums(cuda, S, E, p):
    """a16 (agent :144-167) on the device (dppo_episode_sums): the per-env rows summed in env order
    give the oracle's episode statistics (episodes that start and end inside the rollout, their
    returns, best rewards / act_steps and successes), incl. envs with no finished episode, starts at
    t = 0 and t = S, and episodes of length 1 (not counted)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    rng = np.random.default_rng(S * 1000 + E)
    firsts = (rng.random((S + 1, E)) < p).astype(np.uint8)
    firsts[0, ::2] = 1
    firsts[S, ::3] = 1
    rew = rng.normal(0, 2, (S, E))
    act_steps, thr = 4, 0.3
    out = torch.empty(E, 4, dtype=torch.float64, device=cuda)
    ops.episode_sums(torch.tensor(rew, device=cuda), torch.tensor(firsts, device=cuda), act_steps, thr, out)
    rows = out.cpu().numpy()
    n, tot, best, succ = rows.sum(axis=0)
    ref = O.episode_stats(firsts, rew, act_steps, thr)
    assert int(n) == ref["num_episode_finished"]
    if n:
        assert abs(tot / n - ref["avg_episode_reward"]) <= 1e-12 * max(1.0, abs(ref["avg_episode_reward"]))
        assert abs(best / n - ref["avg_best_reward"]) <= 1e-12 * max(1.0, abs(ref["avg_best_reward"]))
        assert succ / n == ref["success_rate"]


def test_reward_scale_multi_call(cuda):
    import torch
    from diffusionpolicyoptimization_amd import ops
    S, E = 50, 6
    rng = np.random.default_rng(9)
    orc = O.RunningRewardScalerOracle(E)
    ret_state = torch.zeros(E, dtype=torch.float64, device=cuda)
    rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=cuda)
    for it in range(3):
        r = rng.normal(2.0, 3.0, size=(S, E))
        first = (rng.uniform(size=(S, E)) < 0.04).astype(np.uint8)
        ref = orc(r.T, first.T.astype(np.float64)).T
        rt = torch.tensor(r, device=cuda)
        ops.reward_scale(rt, torch.tensor(first, device=cuda), ret_state, rms)
        torch.cuda.synchronize()
        np.testing.assert_allclose(rt.cpu().numpy(), ref, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(rms.cpu().numpy(), [orc.mean, orc.var, orc.count], rtol=1e-10)


@pytest.mark.parametrize("entry", ["dppo_reward_scale", "RunningRewardScaler.scale_", "RunningRewardScaler.__call__"])
def test_reward_scale_matches_reference_goldens(cuda, entry):
    """a18 pinned on the GPU directly: tests/golden/reward_scaling.npz holds outputs of the
    reference's own util/reward_scaling.py (RunningRewardScaler, :42-87, generated by
    tests/golden/make_golden.py) over 4 shapes and 2-4 consecutive calls each. Every call of every
    case goes through the fp64 kernels with the scaler state (ret, mean / var / count) carried
    between calls, through the raw C-ABI entry, the agent's time-major scale_() and the
    reference-signature __call__; outputs, ret and (mean, var, count) at rtol 1e-12."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.reward_scaling import RunningRewardScaler
    g = np.load(os.path.join(ROOT, "tests", "golden", "reward_scaling.npz"))
    ci = 0
    while f"c{ci}_meta" in g:
        E, S, n_calls = (int(x) for x in g[f"c{ci}_meta"])
        ret = torch.zeros(E, dtype=torch.float64, device=cuda)
        rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=cuda)
        sc = RunningRewardScaler(E, device=cuda)
        for k in range(n_calls):
            p = f"c{ci}_k{k}_"
            r, first = g[p + "reward"], g[p + "first"]          # [E, S], the reference's layout
            if entry == "dppo_reward_scale":
                rt = torch.tensor(np.ascontiguousarray(r.T), device=cuda)
                ops.reward_scale(rt, torch.tensor(np.ascontiguousarray(first.T).astype(np.uint8), device=cuda), ret, rms)
                out = rt.cpu().numpy().T
                state = (ret, rms)
            elif entry == "RunningRewardScaler.scale_":
                rt = torch.tensor(np.ascontiguousarray(r.T), device=cuda)
                sc.scale_(rt, torch.tensor(np.ascontiguousarray(first.T).astype(np.uint8), device=cuda))
                out = rt.cpu().numpy().T
                state = (sc.ret, sc.rms)
            else:
                out = sc(reward=r, first=first)
                state = (sc.ret, sc.rms)
            torch.cuda.synchronize()
            np.testing.assert_allclose(out, g[p + "out"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(state[0].cpu().numpy(), g[p + "ret"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(state[1].cpu().numpy(), g[p + "rms"], rtol=1e-12)
        ci += 1
    assert ci == 4


@pytest.mark.parametrize("entry", ["RunningRewardScaler.__call__", "RunningRewardScaler.scale_"])
def test_reward_scale_per_env_matches_reference_goldens(cuda, entry):
    """a18's per_env=True branch (util/reward_scaling.py:51-66) against outputs of the reference's own
    RunningRewardScaler(per_env=True) (tests/golden/reward_scaling_per_env.npz, make_golden.py):
    the state of shape (num_envs,) updated with moments over the ENVS of each time column, NumPy
    broadcasting included — S == E, E == 1 (the state takes S's shape), S == 1 (the output
    broadcasts to [E, L]) — and the shape the reference rejects (E = 4, S = 50) raising ValueError.
    scale_ (in place, time-major) skips the S == 1 < L calls, which cannot be in place."""
    import torch
    from diffusionpolicyoptimization_amd.util.reward_scaling import RunningRewardScaler
    g = np.load(os.path.join(ROOT, "tests", "golden", "reward_scaling_per_env.npz"))
    ci = 0
    checked = 0
    while f"c{ci}_meta" in g:
        E, n_calls = (int(x) for x in g[f"c{ci}_meta"])
        sc = RunningRewardScaler(E, per_env=True, device=cuda)
        for k in range(n_calls):
            p = f"c{ci}_k{k}_"
            r, first = g[p + "reward"], g[p + "first"]
            if p + "raises" in g:
                with pytest.raises(ValueError):
                    sc(reward=r, first=first)
                checked += 1
                break
            if entry == "RunningRewardScaler.scale_" and r.shape[1] == 1 and np.asarray(g[p + "var"]).size > 1:
                with pytest.raises(ValueError):
                    sc.scale_(torch.tensor(np.ascontiguousarray(r.T), device=cuda),
                              torch.tensor(np.ascontiguousarray(first.T).astype(np.uint8), device=cuda))
                break
            if entry == "RunningRewardScaler.__call__":
                out = sc(reward=r, first=first)
            else:
                rt = torch.tensor(np.ascontiguousarray(r.T), device=cuda)
                sc.scale_(rt, torch.tensor(np.ascontiguousarray(first.T).astype(np.uint8), device=cuda))
                out = rt.cpu().numpy().T
            torch.cuda.synchronize()
            assert out.shape == g[p + "out"].shape
            np.testing.assert_allclose(out, g[p + "out"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(sc.ret.cpu().numpy(), g[p + "ret"], rtol=1e-12, atol=1e-12)
            st = sc.ret_rms
            np.testing.assert_allclose(st.mean, np.broadcast_to(g[p + "mean"], st.mean.shape), rtol=1e-12, atol=1e-15)
            assert st.mean.shape == np.asarray(g[p + "mean"]).reshape(-1).shape
            np.testing.assert_allclose(st.var, g[p + "var"], rtol=1e-12)
            np.testing.assert_allclose(st.count, g[p + "count"], rtol=1e-12)
            checked += 1
        ci += 1
    assert ci == 6 and checked >= 8


def test_feistel_bit_exact(cuda):
    from diffusionpolicyoptimization_amd import ops
    for n, seed, ep in [(320000, 42, 0), (1000, 7, 3), (13, 1, 1), (1, 5, 0)]:
        got = ops.feistel_permute(0, n, n, seed, ep, cuda).cpu().numpy()
        ref = PX.feistel_permute(np.arange(n), n, seed, ep)
        assert np.array_equal(got, ref)
        assert np.array_equal(np.sort(got), np.arange(n))


@pytest.mark.parametrize("mode", ["keras", "torch"])
def test_adamw(cuda, mode):
    import torch
    from diffusionpolicyoptimization_amd import ops
    rng = np.random.default_rng(11)
    n = 100003
    p = rng.normal(size=n).astype(np.float32)
    m = np.zeros(n); v = np.zeros(n)
    P, M, V = (torch.tensor(x, dtype=torch.float32, device=cuda) for x in (p, m, v))
    ref = p.astype(np.float64)
    for step in range(1, 4):
        g = rng.normal(size=n).astype(np.float32)
        if mode == "keras":
            ref, m, v = O.keras_adamw_step(ref, g, m, v, step, lr=1e-3, wd=0.004)
            ops.adamw(P, torch.tensor(g, device=cuda), M, V, step, 1e-3, 0.004, 0.9, 0.999, 1e-7, "keras")
        else:
            ref, m, v = O.torch_adamw_step(ref, g, m, v, step, lr=1e-3, wd=0.01)
            ops.adamw(P, torch.tensor(g, device=cuda), M, V, step, 1e-3, 0.01, 0.9, 0.999, 1e-8, "torch")
    torch.cuda.synchronize()
    np.testing.assert_allclose(P.cpu().numpy(), ref, rtol=1e-5, atol=1e-6)


def test_optimizer_step_metrics_tag(cuda):
    """ABI 5: dppo_optimizer_step stores the tag after the metric sums in host-mapped memory; the
    AdamW step equals dppo_adamw's."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", [])
    m = instantiate(cfg.model, device=cuda, seed=0)
    n = m.n_actor
    g = torch.randn(n, device=cuda)
    P0 = m.actor_ft_params.clone()
    M, V = torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    met = torch.arange(16, dtype=torch.float64, device=cuda) * 0.5 + 0.25
    out = ops.MappedDoubles(8)
    for tag in (7, 8):
        ops.optimizer_step(m.dims, m.precision, m.actor_ft_params, g, M, V, 1, 1e-3, 0.004, 0.9, 0.999, 1e-7, "keras",
                           m.actor_ft_params, m.packed_ft, metrics=met, metrics_out=out.address, n_metrics=5,
                           metrics_tag=tag)
        out.wait_tag(5, tag, timeout_s=10.0)
        np.testing.assert_array_equal(out.array[:5], met[:5].cpu().numpy())
        met += 1.0
    torch.cuda.synchronize()
    P1, M1, V1 = P0.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    for _ in range(2):
        ops.adamw(P1, g, M1, V1, 1, 1e-3, 0.004, 0.9, 0.999, 1e-7, "keras")
    torch.cuda.synchronize()
    assert torch.equal(P1, m.actor_ft_params)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_deferred_sampler_tables(cuda, precision):
    """ABI 7: an optimizer step with DPPO_STEP_DEFER_SAMPLER_TABLES packs the actor image without the
    split sampler's tables; the next sampler launch re-derives them on its stream, leaving the image
    byte-identical to a full pack, and samples the same actions as after one. The refresh happens
    once (a second launch finds nothing stale)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      [f"model.precision={precision}"])
    m = instantiate(cfg.model, device=cuda, seed=0)
    n = m.n_actor
    g = torch.randn(n, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3)) * 0.1
    M, V = torch.rand(n, device=cuda) * 1e-3, torch.rand(n, device=cuda) * 1e-6
    P1, M1, V1 = m.actor_ft_params.clone(), M.clone(), V.clone()
    before = m.packed_ft.clone()
    ops.optimizer_step(m.dims, m.precision, m.actor_ft_params, g, M, V, 3, 1e-2, 0.004, 0.9, 0.999, 1e-7, "keras",
                       m.actor_ft_params, m.packed_ft, defer_sampler_tables=True)
    ops.adamw(P1, g, M1, V1, 3, 1e-2, 0.004, 0.9, 0.999, 1e-7, "keras")   # the step's AdamW is dppo_adamw's
    torch.cuda.synchronize()
    assert torch.equal(P1, m.actor_ft_params) and torch.equal(M1, M) and torch.equal(V1, V)
    stale = m.packed_ft.clone()
    full = stale.clone()                 # the same bytes in the gaps between segments
    ops.pack_actor(m.dims, m.actor_ft_params, m.precision, out=full)
    torch.cuda.synchronize()
    assert not torch.equal(stale, full) and not torch.equal(stale, before)   # tables stale, the rest repacked
    cond = torch.rand(64, m.dims.sd, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1)) * 2 - 1
    m._call_id = 0
    a_deferred = m(cond).trajectories.clone()          # refreshes the tables first
    torch.cuda.synchronize()
    assert torch.equal(m.packed_ft, full)
    m.packed_ft.copy_(full)
    m._call_id = 0
    a_full = m(cond).trajectories.clone()
    torch.cuda.synchronize()
    assert torch.equal(a_deferred, a_full)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_l2_deferred_minibatch_and_step(cuda, precision):
    """ABI 8: a minibatch with DPPO_PPO_L2_DEFERRED leaves the actor's l2 gradient factored; formed in
    place (dppo_materialize_l2) it equals the plain minibatch's gradient (up to the dW's float-atomic
    order), and an optimizer step with DPPO_STEP_L2_FROM_PL2 on the factored gradient gives exactly
    the parameters, moments and image of a plain step on the materialised one."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      [f"model.precision={precision}"])
    m = instantiate(cfg.model, device=cuda, seed=0)
    d = m.dims
    N, kf, rows = 64 * 40, d.ft_denoising_steps, 3000
    gen = torch.Generator(device=cuda).manual_seed(0)
    obs = torch.rand(N, d.sd, device=cuda, generator=gen) * 2 - 1
    chains = torch.randn(N, kf + 1, d.xd, device=cuda, generator=gen) * 0.5
    adv = torch.randn(N, device=cuda, generator=gen)
    ret = torch.randn(N, device=cuda, generator=gen)
    lp_old = torch.empty(N, kf, device=cuda)
    ops.logprob(d, m.precision, m.packed_ft, m.sched, obs, chains, want_elem=False, lp_mean=lp_old)
    lp_old += 0.01 * torch.randn(N, kf, device=cuda, generator=gen)
    run = {}
    for deferred in (False, True):
        f = m.bind_minibatch(obs, chains, lp_old, adv, ret, 11, rows, l2_deferred=deferred)
        f(3, 0, rows)
        torch.cuda.synchronize()
        run[deferred] = m.grads.clone()
    g_plain, g_def = run[False], run[True]
    g_mat = g_def.clone()
    ops.materialize_l2(d, m.precision, m.packed_ft, g_mat, m.workspace(rows), rows)
    torch.cuda.synchronize()
    scale = g_plain.abs().max()
    assert (g_mat - g_plain).abs().max() <= 1e-5 * scale, float((g_mat - g_plain).abs().max() / scale)
    na = m.n_actor
    gen2 = torch.Generator(device=cuda).manual_seed(1)
    M0 = torch.rand(na, device=cuda, generator=gen2) * 1e-4
    V0 = torch.rand(na, device=cuda, generator=gen2) * 1e-7
    out = {}
    for virt, g in ((True, g_def), (False, g_mat)):
        P, M, V, img = m.actor_ft_params.clone(), M0.clone(), V0.clone(), m.packed_ft.clone()
        step = ops.BoundOptimizerStep(d, m.precision, P, g[:na], M, V, 0.004, 0.9, 0.999, 1e-7, "keras", P, img,
                                      l2_from_pl2=virt)
        step(2, 1e-3)
        torch.cuda.synchronize()
        out[virt] = (P, M, V, img)
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("net", ["actor", "actor_l2v", "critic"])
@pytest.mark.parametrize("variant", ["fused", "clear"])
def test_fused_optimizer_step_matches_two_launches(cuda, precision, net, variant):
    """ABI 11: an optimizer step with DPPO_STEP_FUSED_PACK | DPPO_STEP_CLEAR_GRADS (one launch: AdamW,
    each element's image slots, the actor's W_OUT / T_OUT slots and the clears by the last workgroup)
    — or DPPO_STEP_CLEAR_GRADS alone (the clears ride on the pack launch) — gives bit-identical
    parameters, moments and image bytes to AdamW + the pack (two launches) once the tables each path
    leaves stale are re-derived (the fused actor step leaves TEMB to its consumers since ABI 12),
    zeroes the range's gradients and the given byte ranges, and leaves its ticket counter reusable
    (three steps in a row on one stream)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      [f"model.precision={precision}"])
    m = instantiate(cfg.model, device=cuda, seed=0)
    d = m.dims
    actor = net != "critic"
    P0 = (m.actor_ft_params if actor else m.critic_params).clone()
    img0 = (m.packed_ft if actor else m.packed_critic).clone()
    n = P0.numel()
    gen = torch.Generator(device=cuda).manual_seed(7)
    G0 = torch.randn(n, device=cuda, generator=gen) * 0.05
    if net == "actor_l2v":   # the factored l2 gradient: pl2 [H][XD] at the l2 region's start, the rest zero
        offs, o = {}, 0
        for name, shape in ops.actor_param_spec(d):
            offs[name] = (o, int(np.prod(shape)))
            o += offs[name][1]
        l2w, nl2 = offs["l2_w"]
        G0[l2w + d.actor_hidden * d.xd:l2w + nl2] = 0
        G0[offs["l2_b"][0]:offs["l2_b"][0] + offs["l2_b"][1]] = 0
    M0 = torch.rand(n, device=cuda, generator=gen) * 1e-4
    V0 = torch.rand(n, device=cuda, generator=gen) * 1e-7
    scratch = torch.full((3, 300), 7.0, dtype=torch.float64, device=cuda)
    out = {}
    for fused in (False, True):
        P, M, V, img, G = P0.clone(), M0.clone(), V0.clone(), img0.clone(), G0.clone()
        packs = (P, img, None, None) if actor else (None, None, P, img)
        step = ops.BoundOptimizerStep(d, m.precision, P, G, M, V, 0.004, 0.9, 0.999, 1e-7, "keras", *packs,
                                      defer_sampler_tables=actor, l2_from_pl2=net == "actor_l2v",
                                      fused_pack=fused and variant == "fused", clear_grads=fused)
        clear = None
        if fused:   # three byte ranges of a scratch buffer, as dppo_ppo_clear_ranges would give
            clear = type("C", (), {})()
            base = scratch.data_ptr()
            ptrs = (ctypes.c_void_p * 4)(base, base + 2400, base + 4800 + 16)
            nb = (ctypes.c_size_t * 4)(8, 2400, 1000)
            clear.args = (ptrs, nb, 3)
        for it in range(3):
            if fused and it:
                G.copy_(G0)
            step(it + 2, 1e-3 * (it + 1), clear=clear)
        if actor:   # the tables each path left stale (ABI 12: the fused actor step leaves TEMB stale too)
            ops.refresh_sampler_tables(img)
        torch.cuda.synchronize()
        out[fused] = (P, M, V, img, G)
    for name, a, b in zip(("params", "m", "v", "image"), out[True][:4], out[False][:4]):
        assert torch.equal(a, b), name
    assert int(torch.count_nonzero(out[True][4])) == 0
    flat = scratch.view(torch.uint8).view(-1)
    assert int(torch.count_nonzero(flat[:8])) == 0 and int(torch.count_nonzero(flat[2400:4800])) == 0
    assert int(torch.count_nonzero(flat[4816:5816])) == 0
    assert bool((flat[8:2400] != 0).any()) and bool((flat[5816:] != 0).any())   # nothing outside the ranges


@pytest.mark.parametrize("net", ["actor", "critic"])
def test_fused_step_clears_after_the_metrics_copy(cuda, net):
    """the fused step's clear ranges are zeroed by its LAST workgroup, after every read of
    the launch, so a range that overlaps the metric sums the step copies out (or its own gradients)
    never zeroes them before they are read: metrics_out holds the sums, the range is zero after."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", [])
    m = instantiate(cfg.model, device=cuda, seed=0)
    d = m.dims
    actor = net == "actor"
    P = (m.actor_ft_params if actor else m.critic_params).clone()
    img = (m.packed_ft if actor else m.packed_critic).clone()
    n = P.numel()
    G = torch.randn(n, device=cuda, generator=torch.Generator(device=cuda).manual_seed(2)) * 0.05
    M, V = torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    met = torch.arange(1, 17, dtype=torch.float64, device=cuda)
    out = ops.MappedDoubles(9)
    packs = (P, img, None, None) if actor else (None, None, P, img)
    step = ops.BoundOptimizerStep(d, m.precision, P, G, M, V, 0.004, 0.9, 0.999, 1e-7, "keras", *packs,
                                  defer_sampler_tables=actor, fused_pack=True, clear_grads=True)
    clear = type("C", (), {})()
    ptrs = (ctypes.c_void_p * 4)(met.data_ptr())
    nb = (ctypes.c_size_t * 4)(16 * 8)
    clear.args = (ptrs, nb, 1)
    step(1, 1e-3, metrics=met, metrics_out=out.address, n_metrics=8, metrics_tag=5, clear=clear)
    out.wait_tag(8, 5)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.array[:8], np.arange(1, 9, dtype=np.float64))
    assert int(torch.count_nonzero(met)) == 0 and int(torch.count_nonzero(G)) == 0
    if actor:
        ops.refresh_sampler_tables(img)
        torch.cuda.synchronize()


def test_value_moments(cuda):
    import torch
    from diffusionpolicyoptimization_amd import ops
    rng = np.random.default_rng(5)
    for n in (1, 777, 32000):
        v = rng.normal(size=n).astype(np.float32)
        r = (v + rng.normal(0, 0.3, n)).astype(np.float32)
        out = ops.MappedDoubles(5)
        ops.value_moments(torch.tensor(v, device=cuda), torch.tensor(r, device=cuda), out.address)
        torch.cuda.synchronize()
        y, d = r.astype(np.float64), r.astype(np.float64) - v.astype(np.float64)
        np.testing.assert_allclose(out.array, [y.sum(), (y * y).sum(), d.sum(), (d * d).sum(), n], rtol=1e-12, atol=1e-9)


def _dedup(bi):
    """(first row, multiplicity) of each distinct sample: the critic's sample-weighted rows."""
    _, first, mult = np.unique(bi, return_index=True, return_counts=True)
    return first, mult


@pytest.mark.parametrize("precision,case,rtol", [("fp32", "perturbed", 2e-3), ("fp32", "ratio1", 2e-3),
                                                  ("bf16", "ratio1", 1e-2), ("bf16", "perturbed", 2e-2),
                                                  ("fp32", "perturbed-ddim", 2e-3), ("fp32", "perturbed-walker", 2e-3),
                                                  ("bf16", "ratio1-walker", 1e-2), ("fp16", "ratio1", 1e-2),
                                                  ("fp16", "ratio1-ddim", 1e-2), ("fp32", "perturbed-narrow", 2e-3),
                                                  ("bf16", "ratio1-narrow", 1e-2), ("fp32", "perturbed-clipv", 2e-3),
                                                  ("bf16", "ratio1-clipv", 1e-2)])
def test_ppo_minibatch_grads(cuda, precision, case, rtol):
    """c_loss forward metrics and gradients of pg_loss + 0.5 v_loss vs the oracle.

    'perturbed': old logprobs = current ones + noise, so ~60% of rows sit on a PPO clip branch;
    exercised in fp32 only, since bf16 rounding flips those discrete branches (a bf16-rounded
    oracle itself moves 10-29% from the f64 one there). 'ratio1': old logprobs are the policy's
    own (the first-epoch situation: ratio == 1, no clip). bf16 is compared against the oracle that
    rounds operands to bf16 at the kernels' rounding points (plain f64 differs by 10-29% here
    because these minibatch sums cancel ~12x and clip branches flip under rounding)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    # DDIM: time-MLP gradient at t = 2j; walker: XD = 24 through the 32-row actor tile; narrow: XD = 8,
    # a width with no instantiation of its own (W_out's gradient through the generic out_back groups)
    # clipv: the clipped value loss (diffusion_ppo.py:110-116, clip_vloss_coef = 0.2) against old values
    # V(obs) + U(-0.4, 0.4), so both of tf.maximum's branches and both sides of the clip occur
    clipv = case.endswith("-clipv")
    dims = {"ddim": HOPPER_DDIM, "walker": WALKER, "narrow": NARROW}.get(case.split("-")[-1], HOPPER)
    case = case.split("-")[0]
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    rng = np.random.default_rng(12)
    N = 40                                  # samples (steps*envs)
    kf = d.ft_denoising_steps
    total = N * kf
    obs = rng.uniform(-1, 1, (N, d.sd)).astype(np.float32)
    chains = (rng.standard_normal((N, kf + 1, d.xd)) * 0.5).astype(np.float32)
    adv = rng.normal(size=N).astype(np.float32)
    ret = rng.normal(size=N).astype(np.float32)
    T = lambda x: torch.tensor(x, device=cuda)
    packf = ops.pack_actor(d, pf, precision)
    lp_ref = O.get_logprobs(to_f64(ft), sched, obs.reshape(N, 1, -1).astype(np.float64),
                            chains.reshape(N, kf + 1, d.horizon_steps, d.action_dim).astype(np.float64), kf, rnd=_rnd(precision))
    lp_ref_mean = np.clip(lp_ref, -5, 2).mean(axis=(1, 2)).reshape(N, kf)
    if case == "perturbed":
        lp_old = (lp_ref_mean + rng.normal(0, 0.02, (N, kf))).astype(np.float32)
        lp_old_gpu = lp_old
        lp_old_ref = lp_old.astype(np.float64)
    else:
        _, lpm = ops.logprob(d, precision, packf, tab, T(obs), T(chains), want_elem=False)
        lp_old_gpu = lpm.cpu().numpy()
        lp_old_ref = lp_ref_mean
    seed, epoch, start, rows = 99, 1, 37, 150
    perm = PX.feistel_permute(np.arange(start, start + rows), total, seed, epoch)
    bi, di = perm // kf, perm % kf
    oldv, cv = None, None
    if clipv:
        v_now = O.critic_forward(to_f64(critic), obs.reshape(N, 1, -1).astype(np.float64), rnd=_rnd(precision))[0][:, 0]
        oldv = (v_now + rng.uniform(-0.4, 0.4, N)).astype(np.float32)
        cv = 0.2
    metrics_ref, ga_ref, gc_ref = O.c_loss(
        to_f64(ft), to_f64(critic), sched, obs[bi].reshape(rows, 1, -1).astype(np.float64),
        chains[bi, di].reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64), chains[bi, di + 1].reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64),
        di, ret[bi].astype(np.float64), None if oldv is None else oldv[bi].astype(np.float64), adv[bi].astype(np.float64),
        lp_old_ref[bi, di], kf, rnd=_rnd(precision), critic_dedup=_dedup(bi), clip_vloss_coef=cv)
    na = ops.spec_count(ops.actor_param_spec(d))
    nc = ops.spec_count(ops.critic_param_spec(d))
    grads = torch.zeros(na + nc, dtype=torch.float32, device=cuda)
    metrics = torch.zeros(16, dtype=torch.float64, device=cuda)
    ws = ops.ppo_workspace(d, precision, rows, cuda)
    oldv_dev = T(oldv) if clipv else None
    hp = ops.ppo_hparams(global_rows=rows, clip_vloss_coef=cv, old_values=oldv_dev)
    ops.ppo_minibatch(d, precision, hp, packf, ops.pack_critic(d, pc, precision), pf, tab,
                      T(obs), T(chains), T(lp_old_gpu), T(adv), T(ret), seed, epoch, start, rows, ws, grads, metrics)
    torch.cuda.synchronize()
    m = metrics.cpu().numpy() / rows
    assert abs(m[0] - metrics_ref["pg_loss"]) < rtol * (abs(metrics_ref["pg_loss"]) + 1e-2)
    assert abs(m[1] - metrics_ref["v_loss"]) < rtol * (abs(metrics_ref["v_loss"]) + 1e-2)
    assert abs(m[2] - metrics_ref["approx_kl"]) < rtol * 10 * (abs(metrics_ref["approx_kl"]) + 1e-4)
    assert abs(m[3] - metrics_ref["clipfrac"]) <= (0.0 if case == "ratio1" else 0.02)
    g = grads.cpu().numpy()
    ga = ops.unflatten_params(ops.actor_param_spec(d), g[:na])
    gc = ops.unflatten_params(ops.critic_param_spec(d), g[na:])
    errs = {}
    for name, ref in list(ga_ref.items()):
        errs[name] = np.abs(ga[name] - ref).max() / (np.abs(ref).max() + 1e-12)
    for name, ref in gc_ref.items():
        errs["critic." + name] = np.abs(gc[name] - ref).max() / (np.abs(ref).max() + 1e-12)
    bad = {k: float(v) for k, v in errs.items() if not v < rtol}
    assert not bad, (bad, {k: float(v) for k, v in errs.items()})


@pytest.mark.parametrize("precision,rtol", [("fp32", 2e-3), ("bf16", 1e-2), ("fp16", 1e-2)])
@pytest.mark.parametrize("dims", [HOPPER, WALKER], ids=["hopper", "walker"])
def test_pretrain_loss_grads(cuda, precision, rtol, dims):
    """§8(f) row 3: p_losses / q_sample (diffusion.py:179-202) through the TRAIN row tile
    (dppo_pretrain_minibatch): loss and every actor gradient vs the oracle, t over all K = 20 steps
    (bucket sums of the time-MLP gradient over 20 t's), ragged rows. bf16 compares against the
    oracle rounding operands at the kernels' rounding points."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    rng = np.random.default_rng(21)
    rows = 150
    K = d.denoising_steps
    x0 = rng.uniform(-1, 1, (rows, d.xd)).astype(np.float32)
    cond = rng.uniform(-1, 1, (rows, d.sd)).astype(np.float32)
    t = rng.integers(0, K, rows).astype(np.int32)
    noise = rng.standard_normal((rows, d.xd)).astype(np.float32)
    loss_ref, g_ref = O.p_losses(to_f64(ft), sched, x0.reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64),
                                 cond.reshape(rows, d.cond_steps, d.obs_dim).astype(np.float64), t,
                                 noise.reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64),
                                 rnd=_rnd(precision))
    T = lambda x: torch.tensor(x, device=cuda)
    na = ops.spec_count(ops.actor_param_spec(d))
    grads = torch.zeros(na, dtype=torch.float32, device=cuda)
    metrics = torch.zeros(16, dtype=torch.float64, device=cuda)
    ws = ops.ppo_workspace(d, precision, rows, cuda)
    loss = ops.pretrain_minibatch(d, precision, ops.pack_actor(d, pf, precision), pf, tab, T(ops.q_sched_table(sched)),
                                  T(x0), T(cond), T(t), T(noise), ws, grads, metrics)
    torch.cuda.synchronize()
    assert abs(float(loss) - loss_ref) < rtol * loss_ref
    ga = ops.unflatten_params(ops.actor_param_spec(d), grads.cpu().numpy())
    errs = {k: float(np.abs(ga[k] - ref).max() / (np.abs(ref).max() + 1e-12)) for k, ref in g_ref.items()}
    bad = {k: v for k, v in errs.items() if not v < rtol}
    assert not bad, (bad, errs)


def test_adv_stats_all_matches_per_minibatch(cuda):
    """dppo_ppo_adv_stats_all (every minibatch of an update phase in one launch) == one
    dppo_ppo_adv_stats call per minibatch, ragged last minibatch included."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    rng = np.random.default_rng(4)
    N, kf = 97, 10
    total = N * kf
    adv = torch.tensor(rng.normal(size=N).astype(np.float32), device=cuda)
    rows_full, n_batch, n_ep, seed, ep0 = 200, 5, 3, 77, 3000
    allst = torch.zeros(n_ep * n_batch, 3, dtype=torch.float64, device=cuda)
    ops.ppo_adv_stats_all(adv, total, kf, seed, ep0, n_ep, rows_full, n_batch, allst)
    one = torch.zeros(3, dtype=torch.float64, device=cuda)
    for e in range(n_ep):
        for b in range(n_batch):
            start = b * rows_full
            rows = min(rows_full, total - start)
            ops.ppo_adv_stats(adv, total, kf, seed, ep0 + e, start, rows, one)
            torch.testing.assert_close(allst[e * n_batch + b], one, rtol=1e-12, atol=1e-9)


def test_logprob_pass_full_size(cuda):
    """The old-log-prob pass (a10 + c_loss:50-59, agent :209-229) at the bench's size: S*E =
    500 x 64 = 32,000 samples (320,000 rows) in one launch, fp32; 256 random samples checked
    against the oracle (element log-probs and the clipped per-row mean)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    n, kf = 32000, d.ft_denoising_steps
    g = torch.Generator(device=cuda).manual_seed(5)
    obs = torch.rand(n, d.sd, device=cuda, generator=g) * 2 - 1
    chains = torch.randn(n, kf + 1, d.xd, device=cuda, generator=g) * 0.5
    packf = ops.pack_actor(d, pf, "fp32")
    lpe, lpm = ops.logprob(d, "fp32", packf, tab, obs, chains, want_elem=True, want_mean=True)
    torch.cuda.synchronize()
    pick = np.random.default_rng(3).choice(n, 256, replace=False)
    o, c = obs.cpu().numpy()[pick], chains.cpu().numpy()[pick]
    ref = O.get_logprobs(to_f64(ft), sched, o.reshape(-1, 1, d.sd).astype(np.float64),
                         c.reshape(-1, kf + 1, d.horizon_steps, d.action_dim).astype(np.float64), kf)
    got = lpe.view(n, kf, d.xd).cpu().numpy()[pick].reshape(ref.shape)
    assert np.abs(got - ref).max() < 1e-3, np.abs(got - ref).max()
    ref_m = np.clip(ref, -5, 2).mean(axis=(1, 2)).reshape(-1, kf)
    assert np.abs(lpm.cpu().numpy()[pick] - ref_m).max() < 1e-4


@pytest.mark.parametrize("precision,dims", [("fp32", HOPPER), ("bf16", HOPPER), ("fp16", HOPPER),
                                            ("bf16", WALKER), ("fp32", WALKER), ("fp16", HOPPER_DDIM)],
                         ids=["fp32-hopper", "bf16-hopper-config2", "fp16-hopper", "bf16-walker-config3-4",
                              "fp32-walker", "fp16-ddim-config5"])
def test_ppo_minibatch_full_size(cuda, precision, dims):
    """dppo_ppo_minibatch at the bench's minibatch, b = 50,000 rows (782 64-row actor tiles at
    hopper dims; at walker2d / halfcheetah dims, XD = 24, the actor runs 32-row tiles: 1,563 of
    them; split-K dW over all rows), over a 64,000-row rollout, for every per-GPU shard shape of
    BASELINE configs 2-5 (config 5: DDIM, 10 rows over K = 20, fp16). The full-size launch is
    checked through a size-independent property and the oracle:
      * linearity: the loss is a mean over rows, so the gradient and metric sums of the full
        launch equal the sum over 25 disjoint 2,000-row slices of the same rows (row_index), each
        launched with global_rows = 50,000 and the full minibatch's advantage moments;
      * one of those slices against the oracle (c_loss with denom = 50,000 and the full
        minibatch's advantage mean / std)."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(dims, cuda)
    N, kf, b, perm_seed, epoch = 6400, d.ft_denoising_steps, 50000, 77, 3
    rng = np.random.default_rng(21)
    obs = rng.uniform(-1, 1, (N, d.sd)).astype(np.float32)
    chains = (rng.standard_normal((N, kf + 1, d.xd)) * 0.5).astype(np.float32)
    adv = rng.normal(size=N).astype(np.float32)
    ret = rng.normal(size=N).astype(np.float32)
    T = lambda x: torch.tensor(x, device=cuda)
    packf, packc = ops.pack_actor(d, pf, precision), ops.pack_critic(d, pc, precision)
    _, lpm = ops.logprob(d, precision, packf, tab, T(obs), T(chains), want_elem=False)
    # fp32: perturbed old log-probs (rows on both PPO clip branches); bf16: the policy's own (ratio 1),
    # since bf16 rounding flips clip branches (see test_ppo_minibatch_grads)
    noise = rng.normal(0, 0.01, (N, kf)) if precision == "fp32" else 0.0
    lp_old = (lpm.cpu().numpy() + noise).astype(np.float32)
    args = (T(obs), T(chains), T(lp_old), T(adv), T(ret))
    na = ops.spec_count(ops.actor_param_spec(d))
    nc = ops.spec_count(ops.critic_param_spec(d))
    stats = torch.zeros(3, dtype=torch.float64, device=cuda)
    ops.ppo_adv_stats(args[3], N * kf, kf, perm_seed, epoch, 0, b, stats)
    hp = ops.ppo_hparams(global_rows=b)

    def run(rows, row_index=None, start=0):
        grads = torch.zeros(na + nc, dtype=torch.float32, device=cuda)
        met = torch.zeros(16, dtype=torch.float64, device=cuda)
        ops.ppo_minibatch(d, precision, hp, packf, packc, pf, tab, *args, perm_seed, epoch, start, rows,
                          ops.ppo_workspace(d, precision, rows, cuda), grads, met, adv_stats=stats,
                          row_index=row_index)
        torch.cuda.synchronize()
        return grads.cpu().numpy().astype(np.float64), met.cpu().numpy()[:5]

    g_full, m_full = run(b)
    assert np.isfinite(g_full).all()
    perm = ops.feistel_permute(0, b, N * kf, perm_seed, epoch, cuda)
    g_sum, m_sum = np.zeros_like(g_full), np.zeros(5)
    g_slices = []
    for k in range(25):
        g, m = run(2000, row_index=perm, start=2000 * k)
        g_sum += g
        m_sum += m
        g_slices.append(g)
    # the critic runs once per distinct sample with its multiplicity as the row weight; a sample's
    # multiplicity in a 2,000-row slice differs from the full minibatch's, and with 2-byte operands
    # the weighted gradient seed is rounded once per sample (bf16(w dv) vs a sum of smaller ones):
    # rounding-level differences, so the critic half gets its own bound there
    for lo, hi, tol_g in ((0, na, 1e-5 if precision == "fp32" else 1e-4),
                          (na, na + nc, 1e-5 if precision == "fp32" else 1e-3)):
        rel = np.abs(g_sum[lo:hi] - g_full[lo:hi]).max() / np.abs(g_full[lo:hi]).max()
        assert rel < tol_g, (lo, rel)
    # metric sums (pg, v, approx_kl, clipfrac, ratio) over 50,000 rows: fp32 accumulation order;
    # approx_kl is ~0 at ratio 1 (bf16 case), so it gets an absolute bound. The 2,000-row slices run
    # 32-row actor tiles (a sub-round minibatch), whose out-layer sums in another order: with 2-byte
    # operands that moves log-prob ulps, and the pg sum over 50,000 rows by ~6e-5 relative
    tol = 1e-5 if precision == "fp32" else 2e-4
    np.testing.assert_allclose(m_sum, m_full, rtol=tol, atol=tol)
    # slice 7 against the oracle
    rows = perm.cpu().numpy()[14000:16000]
    bi, di = rows // kf, rows % kf
    st = stats.cpu().numpy()
    mean = st[1] / st[0]
    std = np.sqrt(max(st[2] / st[0] - mean * mean, 0.0))
    met_ref, ga, gc = O.c_loss(
        to_f64(ft), to_f64(critic), sched, obs[bi].reshape(-1, 1, d.sd).astype(np.float64),
        chains[bi, di].reshape(-1, d.horizon_steps, d.action_dim).astype(np.float64),
        chains[bi, di + 1].reshape(-1, d.horizon_steps, d.action_dim).astype(np.float64), di,
        ret[bi].astype(np.float64), None, adv[bi].astype(np.float64), lp_old[bi, di].astype(np.float64), kf,
        rnd=_rnd(precision), adv_mean_std=(mean, std), denom=b, critic_dedup=_dedup(bi))
    g_ref = np.concatenate([ops.flatten_params(ops.actor_param_spec(d), ga).astype(np.float64),
                            ops.flatten_params(ops.critic_param_spec(d), gc).astype(np.float64)])
    g7 = g_slices[7]
    tol = 5e-3 if precision == "fp32" else 1e-2
    for lo, hi, name in ((0, na, "actor"), (na, na + nc, "critic")):
        err = np.abs(g7[lo:hi] - g_ref[lo:hi]).max() / np.abs(g_ref[lo:hi]).max()
        assert err < tol, (name, err)


def test_fp16_small_minibatch_large_returns_stays_finite(cuda):
    """the fp16 backward seed is scale / global_rows x the per-row gradient; with a
    fixed 4096 a 24-row minibatch with value errors ~1e3 overflowed fp16. The scale is now the
    largest power of two <= min(4096, global_rows): finite gradients, matching the oracle."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER, cuda)
    rng = np.random.default_rng(4)
    N, kf, rows = 12, d.ft_denoising_steps, 24
    obs = rng.uniform(-1, 1, (N, d.sd)).astype(np.float32)
    chains = (rng.standard_normal((N, kf + 1, d.xd)) * 0.5).astype(np.float32)
    adv = rng.normal(size=N).astype(np.float32)
    ret = (rng.normal(size=N) * 1000.0).astype(np.float32)
    T = lambda x: torch.tensor(x, device=cuda)
    packf = ops.pack_actor(d, pf, "fp16")
    _, lpm = ops.logprob(d, "fp16", packf, tab, T(obs), T(chains), want_elem=False)
    lp_old = lpm.cpu().numpy()
    na = ops.spec_count(ops.actor_param_spec(d))
    nc = ops.spec_count(ops.critic_param_spec(d))
    grads = torch.zeros(na + nc, dtype=torch.float32, device=cuda)
    met = torch.zeros(16, dtype=torch.float64, device=cuda)
    seed, epoch = 3, 0
    ops.ppo_minibatch(d, "fp16", ops.ppo_hparams(global_rows=rows), packf, ops.pack_critic(d, pc, "fp16"), pf, tab,
                      T(obs), T(chains), T(lp_old), T(adv), T(ret), seed, epoch, 0, rows,
                      ops.ppo_workspace(d, "fp16", rows, cuda), grads, met)
    torch.cuda.synchronize()
    g = grads.cpu().numpy()
    assert np.isfinite(g).all() and np.isfinite(met.cpu().numpy()).all()
    perm = PX.feistel_permute(np.arange(rows), N * kf, seed, epoch)
    bi, di = perm // kf, perm % kf
    _, ga, gc = O.c_loss(to_f64(ft), to_f64(critic), sched, obs[bi].reshape(rows, 1, -1).astype(np.float64),
                         chains[bi, di].reshape(rows, 4, 3).astype(np.float64),
                         chains[bi, di + 1].reshape(rows, 4, 3).astype(np.float64), di, ret[bi].astype(np.float64),
                         None, adv[bi].astype(np.float64), lp_old[bi, di].astype(np.float64), kf, rnd=O.round_fp16,
                         critic_dedup=_dedup(bi))
    gcrit = ops.unflatten_params(ops.critic_param_spec(d), g[na:])
    for k in ("l1_w", "out_w", "in_w"):
        rel = np.abs(gcrit[k] - gc[k]).max() / (np.abs(gc[k]).max() + 1e-12)
        assert rel < 2e-2, (k, rel)


@pytest.mark.parametrize("precision,rtol", [("fp32", 2e-3), ("fp16", 3e-2)])
def test_learn_eta_gradient_matches_oracle(cuda, precision, rtol):
    """§8(f) row 4, learnable DDIM eta (PARITY UNPINNED: the reference's eta module is absent; the
    oracle's derivative is pinned to central differences of its own loss, test_oracle.py): with
    DPPO_PPO_LEARN_ETA the actor's row tiles add d loss / d eta into metrics[8]; checked against the
    oracle at eta = 0.6 (rows on both the free and the min_logprob_std-clipped std branch), 'perturbed'
    old log-probs (fp32) or ratio 1 (fp16). The other metrics and gradients are those of the
    fixed-eta minibatch (test_ppo_minibatch_grads); the flag must not change them."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    eta = 0.6
    d, base, ft, critic, sched, tab, pb, pf, pc = _setup(HOPPER_DDIM, cuda, eta=eta)
    rng = np.random.default_rng(12)
    N, kf = 40, d.ft_denoising_steps
    total = N * kf
    obs = rng.uniform(-1, 1, (N, d.sd)).astype(np.float32)
    chains = (rng.standard_normal((N, kf + 1, d.xd)) * 0.5).astype(np.float32)
    adv = rng.normal(size=N).astype(np.float32)
    ret = rng.normal(size=N).astype(np.float32)
    T = lambda x: torch.tensor(x, device=cuda)
    packf = ops.pack_actor(d, pf, precision)
    lp_ref = O.get_logprobs(to_f64(ft), sched, obs.reshape(N, 1, -1).astype(np.float64),
                            chains.reshape(N, kf + 1, d.horizon_steps, d.action_dim).astype(np.float64), kf,
                            rnd=_rnd(precision))
    lp_ref_mean = np.clip(lp_ref, -5, 2).mean(axis=(1, 2)).reshape(N, kf)
    if precision == "fp32":
        lp_old_gpu = (lp_ref_mean + rng.normal(0, 0.02, (N, kf))).astype(np.float32)
        lp_old_ref = lp_old_gpu.astype(np.float64)
    else:
        _, lpm = ops.logprob(d, precision, packf, tab, T(obs), T(chains), want_elem=False)
        lp_old_gpu = lpm.cpu().numpy()
        lp_old_ref = lp_ref_mean
    seed, epoch, start, rows = 99, 1, 37, 150
    perm = PX.feistel_permute(np.arange(start, start + rows), total, seed, epoch)
    bi, di = perm // kf, perm % kf
    mref, _, _ = O.c_loss(
        to_f64(ft), to_f64(critic), sched, obs[bi].reshape(rows, 1, -1).astype(np.float64),
        chains[bi, di].reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64),
        chains[bi, di + 1].reshape(rows, d.horizon_steps, d.action_dim).astype(np.float64),
        di, ret[bi].astype(np.float64), None, adv[bi].astype(np.float64), lp_old_ref[bi, di], kf,
        rnd=_rnd(precision), critic_dedup=_dedup(bi), eta_grad=True)
    na, nc = ops.spec_count(ops.actor_param_spec(d)), ops.spec_count(ops.critic_param_spec(d))
    packc = ops.pack_critic(d, pc, precision)
    outs = []
    for learn in (True, False):
        grads = torch.zeros(na + nc, dtype=torch.float32, device=cuda)
        metrics = torch.zeros(16, dtype=torch.float64, device=cuda)
        ops.ppo_minibatch(d, precision, ops.ppo_hparams(global_rows=rows, learn_eta=learn), packf, packc, pf, tab,
                          T(obs), T(chains), T(lp_old_gpu), T(adv), T(ret), seed, epoch, start, rows,
                          ops.ppo_workspace(d, precision, rows, cuda), grads, metrics)
        torch.cuda.synchronize()
        outs.append((grads.cpu().numpy(), metrics.cpu().numpy()))
    (g1, m1), (g0, m0) = outs
    ref = mref["d_eta"]
    assert abs(ref) > 1e-3
    assert abs(m1[8] - ref) <= rtol * abs(ref), (m1[8], ref)
    assert m0[8] == 0.0
    np.testing.assert_allclose(m1[:5], m0[:5], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(g1, g0, rtol=1e-4, atol=1e-6 * np.abs(g0).max())


def test_eta_step_matches_numpy(cuda):
    """dppo_eta_step: Keras AdamW on the eta logit from metrics[8] x d eta / d logit, then the DDIM
    table's eta columns (c2, c3, logvar) for the new eta equal ddim_buffers at that eta (fp32, the
    same order of operations: within 2 ulp), the other columns untouched; a refresh (metrics None)
    leaves the logit alone."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddim_buffers
    lo, hi, base = 0.1, 1.0, 0.5
    logit = O.eta_logit_init(base, lo, hi)
    dd = ddim_buffers(20, 10, base)
    tab = torch.tensor(ops.sched_table(dd), device=cuda)
    tab0 = tab.clone()
    eb = torch.tensor(ops.ddim_eta_base(dd), device=cuda)
    st = torch.tensor([logit, 0.0, 0.0], dtype=torch.float32, device=cuda)
    met = torch.zeros(16, dtype=torch.float64, device=cuda)
    out = torch.zeros(1, dtype=torch.float32, device=cuda)
    p, m, v = np.float64(np.float32(logit)), 0.0, 0.0
    for step, g_eta in enumerate((0.7, -0.3, 1.1), start=1):
        met[8] = g_eta
        ops.eta_step(st, met, step, 1e-2, 0.004, lo, hi, eb, tab, eta_out=out)
        torch.cuda.synchronize()
        g = g_eta * 0.5 * (hi - lo) * (1 - np.tanh(p) ** 2)
        p, m, v = O.keras_adamw_step(np.array([p]), np.array([g]), np.array([m]), np.array([v]), step, lr=1e-2, wd=0.004)
        p, m, v = float(p[0]), float(m[0]), float(v[0])
        got = st.cpu().numpy()
        np.testing.assert_allclose(got, [p, m, v], rtol=1e-5, atol=1e-7)
        e = float(out.item())
        assert abs(e - O.eta_from_logit(float(got[0]), lo, hi)) < 1e-6
        ref = ops.sched_table(ddim_buffers(20, 10, np.float32(e)))
        t = tab.cpu().numpy()
        np.testing.assert_array_equal(t[:, [0, 1, 5, 6, 7]], tab0.cpu().numpy()[:, [0, 1, 5, 6, 7]])
        np.testing.assert_allclose(t[:, 2:5], ref[:, 2:5], rtol=3e-7, atol=1e-7)
    before = st.clone()
    ops.eta_step(st, None, 0, 0.0, 0.0, lo, hi, eb, tab, eta_out=out)
    torch.cuda.synchronize()
    assert torch.equal(before, st)

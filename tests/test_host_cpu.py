"""Host-side checks that need no GPU: the C-ABI library loads and exports exactly what
include/dppo.h declares, its host-only queries and argument validation, the native env stepper
against its NumPy specification, and the LR schedules."""
import ctypes
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dppo.h")


@pytest.fixture(scope="module")
def lib():
    from diffusionpolicyoptimization_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "diffusionpolicyoptimization_amd", "csrc"), "-j8"],
                       check=True)
    return _lib.load()


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"DPPO_API\s+[\w\s\*]+?\b(dppo_\w+)\s*\(", src)))


def test_header_and_binding_agree():
    from diffusionpolicyoptimization_amd import _lib
    names = _declared()
    assert len(names) >= 20
    assert names == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    nm = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dppo_\w+)", nm))
    assert set(_declared()) <= exported
    assert exported <= set(_declared()), f"undeclared exports: {exported - set(_declared())}"
    assert lib.dppo_abi_version() == 15


def test_env_library_exports_exactly_its_header():
    """libdppo_env.so (the wrapper stack, its thread pool, the synthetic stepper) exports exactly the
    functions include/dppo_env.h declares."""
    from diffusionpolicyoptimization_amd.env.synthetic import _ENV_LIB
    if not os.path.exists(_ENV_LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "diffusionpolicyoptimization_amd", "csrc"),
                        "../lib/libdppo_env.so"], check=True)
    src = open(os.path.join(ROOT, "include", "dppo_env.h")).read()
    declared = set(re.findall(r"^[\w\s\*]+?\b(dppo_\w+)\s*\(", src, flags=re.M))
    assert len(declared) >= 25
    nm = subprocess.run(["nm", "-D", "--defined-only", _ENV_LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dppo_\w+)", nm))
    assert declared == exported, (declared ^ exported)
    L = ctypes.CDLL(_ENV_LIB)
    assert L.dppo_lowdim_abi() == 2 and L.dppo_env_abi() == 3


def test_host_queries_match_python_layout(lib):
    from diffusionpolicyoptimization_amd import ops
    for d in (ops.ModelDims(), ops.ModelDims(obs_dim=17, action_dim=6), ops.ModelDims(actor_hidden=256)):
        c = d.c()
        assert lib.dppo_actor_param_count(ctypes.byref(c)) == ops.spec_count(ops.actor_param_spec(d))
        assert lib.dppo_critic_param_count(ctypes.byref(c)) == ops.spec_count(ops.critic_param_spec(d))
        for prec in (0, 1):
            nb = lib.dppo_actor_packed_bytes(ctypes.byref(c), prec)
            assert nb > 0 and nb % 256 == 0
            # bf16 images hold half the bytes of fp32 in the weight segments
        assert lib.dppo_actor_packed_bytes(ctypes.byref(c), 1) < lib.dppo_actor_packed_bytes(ctypes.byref(c), 0)
    assert lib.dppo_reward_scale_workspace_doubles(500, 64) > 0


def test_ppo_clear_ranges_are_what_each_part_zeroes(lib):
    """ABI 11: dppo_ppo_clear_ranges (host-side address arithmetic, no device work) reports the
    non-gradient ranges a minibatch part zeroes: the actor (part 1 / 4) metrics 0 and 2..15 and its
    workspace accumulators, the critic (part 2) metric 1 and its own; all inside the workspace or the
    metrics buffer, 4-B aligned, disjoint between the halves."""
    import torch
    from diffusionpolicyoptimization_amd import ops
    d = ops.ModelDims()
    rows = 6250
    ws = torch.empty(ops._workspace_bytes(d, 1, rows), dtype=torch.uint8)
    met = torch.zeros(16, dtype=torch.float64)
    w0, w1, m0 = ws.data_ptr(), ws.data_ptr() + ws.numel(), met.data_ptr()
    got = {p: ops.ClearRanges(d, "bf16", rows, ws, met, p).ranges() for p in (1, 2, 3, 4)}
    assert got[1] == got[4] and len(got[1]) == 3 and len(got[2]) == 2 and len(got[3]) == 3
    assert got[1][:2] == [(m0, 8), (m0 + 16, 112)] and got[2][0] == (m0 + 8, 8)
    assert got[3][0] == (m0, 128)
    spans = []
    for p in (1, 2):
        for a, n in got[p]:
            assert a % 4 == 0 and n % 4 == 0 and n > 0
            assert (m0 <= a and a + n <= m0 + 128) or (w0 <= a and a + n <= w1)
            spans.append((a, a + n))
    spans.sort()
    assert all(e <= s for (_, e), (s, _) in zip(spans, spans[1:]))   # actor and critic ranges disjoint
    with pytest.raises(Exception):
        ops.ClearRanges(d, "bf16", rows, ws, met, 5)


@pytest.mark.parametrize("field,value,msg", [("actor_hidden", 100, "actor_hidden"), ("time_dim", 3, "time_dim"),
                                             ("ft_denoising_steps", 30, "ft_denoising_steps"),
                                             ("action_dim", 9, "horizon_steps*action_dim")])
def test_invalid_dims_fail_loudly_before_any_device_work(lib, field, value, msg):
    from diffusionpolicyoptimization_amd import ops
    d = ops.ModelDims(**{field: value})
    c = d.c()
    assert lib.dppo_actor_param_count(ctypes.byref(c)) == 0
    rc = lib.dppo_sample(ctypes.byref(c), 0, None, None, None, None, 4, None, None, 0, 0, 0, 0, 0.1, 3.0, 1.0,
                         None, None, None)
    assert rc == 1
    assert msg in lib.dppo_last_error().decode()


def test_missing_library_raises(tmp_path):
    from diffusionpolicyoptimization_amd import _lib
    saved = _lib._lib
    _lib._lib = None
    try:
        with pytest.raises(_lib.DppoError, match="no CPU fallback"):
            _lib.load(str(tmp_path / "libdppo_hip.so"))
    finally:
        _lib._lib = saved


def test_native_env_matches_numpy_spec():
    from diffusionpolicyoptimization_amd.env.synthetic import SyntheticLocomotionVecEnv, _native
    if _native() is None:
        subprocess.run(["make", "-C", os.path.join(ROOT, "diffusionpolicyoptimization_amd", "csrc"), "-j8"],
                       check=True)
    E, Do, Da = 7, 11, 3
    envs = [SyntheticLocomotionVecEnv(E, Do, Da, act_steps=4, max_episode_steps=40, family_seed=2, native=nat)
            for nat in (True, False)]
    assert envs[0].native is not None and envs[1].native is None
    for e in envs:
        e.seed(range(100, 100 + E))
    o0, o1 = envs[0].reset_arg(), envs[1].reset_arg()
    np.testing.assert_allclose(o0["state"], o1["state"])
    rng = np.random.default_rng(0)
    n_trunc = 0
    for _ in range(25):
        a = rng.normal(0, 0.8, (E, 4, Da)).astype(np.float32)
        r0 = envs[0].step(a)
        r1 = envs[1].step(a)
        np.testing.assert_allclose(r0[0]["state"], r1[0]["state"], atol=3e-6)
        np.testing.assert_allclose(r0[1], r1[1], atol=3e-6)
        np.testing.assert_array_equal(r0[2], r1[2])
        np.testing.assert_array_equal(r0[3], r1[3])
        n_trunc += int(r0[3].sum())
    assert n_trunc == 2 * E  # 40 sub-steps = 10 chunks; 25 chunks cross two truncations


def test_gated_env_step_publishes_only_without_resets():
    """dppo_env_step_gated: waits for the done counter, steps like the ungated stepper, and
    publishes go only when no env needs a host-side reset (else the caller resets, then publishes)."""
    import ctypes

    from diffusionpolicyoptimization_amd.env.synthetic import SyntheticLocomotionVecEnv, _native
    if _native() is None:
        subprocess.run(["make", "-C", os.path.join(ROOT, "diffusionpolicyoptimization_amd", "csrc"), "-j8"],
                       check=True)
    E, Do, Da = 5, 11, 3
    envs = [SyntheticLocomotionVecEnv(E, Do, Da, act_steps=4, max_episode_steps=12, family_seed=1) for _ in range(2)]
    for e in envs:
        e.seed(range(E))
        e.reset_arg()
    ctr = np.zeros(32, dtype=np.uint32)        # done at [0], go at [16]
    done_p = ctypes.c_void_p(ctr.ctypes.data)
    go_p = ctypes.c_void_p(ctr.ctypes.data + 64)
    obs = [np.zeros((E, 1, Do), np.float32) for _ in range(2)]
    rng = np.random.default_rng(1)
    pubs = []
    for i in range(5):                          # 12 sub-steps = 3 chunks: step 2 truncates every env
        a = rng.normal(0, 0.5, (E, 4, Da)).astype(np.float32)
        ctr[0] = i + 1                          # the "device" has finished step i
        g = envs[0].step(a, obs_out=obs[0], gate=("go", done_p, ctypes.c_uint32(i + 1), go_p, ctypes.c_uint32(i + 2),
                                                  ctypes.c_double(1.0)))
        r = envs[1].step(a, obs_out=obs[1])
        np.testing.assert_array_equal(obs[0], obs[1])
        np.testing.assert_array_equal(g[1], r[1])
        np.testing.assert_array_equal(g[3], r[3])
        pubs.append(envs[0].published)
        if envs[0].published:
            assert ctr[16] == i + 2
    assert pubs == [True, True, False, True, True]
    with pytest.raises(RuntimeError, match="did not finish"):     # done never reaches the target
        envs[0].step(a, obs_out=obs[0], gate=("go", done_p, ctypes.c_uint32(99), None, ctypes.c_uint32(0),
                                              ctypes.c_double(0.01)))
    ctr[0] = 0x80000000                                           # the device's go-wait timed out
    with pytest.raises(RuntimeError, match="timed out"):
        envs[0].step(a, obs_out=obs[0], gate=("go", done_p, ctypes.c_uint32(1), None, ctypes.c_uint32(0),
                                              ctypes.c_double(1.0)))


def test_gated_env_step_tagged_publishes_granules():
    """dppo_env_step_gated_tagged: the stepper polls the launch's actions as tagged granules
    {tag << 32 | fp32 bits} (decoding them into the actions buffer), steps, and publishes the
    observation as tagged granules (what the sampler polls, dppo_rollout_enqueue_tagged). A stale
    action tag with the done counter's timeout bit set fails with -2; with no bit, the host timeout
    fails with -1."""
    import ctypes

    from diffusionpolicyoptimization_amd.env.synthetic import SyntheticLocomotionVecEnv, _native
    if _native() is None:
        subprocess.run(["make", "-C", os.path.join(ROOT, "diffusionpolicyoptimization_amd", "csrc"), "-j8"],
                       check=True)
    E, Do, Da = 5, 11, 3
    envs = [SyntheticLocomotionVecEnv(E, Do, Da, act_steps=4, max_episode_steps=12, family_seed=1) for _ in range(2)]
    for e in envs:
        e.seed(range(E))
        e.reset_arg()
    ctr = np.zeros(16, dtype=np.uint32)
    done_p = ctypes.c_void_p(ctr.ctypes.data)
    tagged = np.zeros(E * Do, np.uint64)
    tag_p = ctypes.c_void_p(tagged.ctypes.data)
    obs = [np.zeros((E, 1, Do), np.float32) for _ in range(2)]
    rng = np.random.default_rng(1)
    pubs = []
    act_t = np.zeros(E * 4 * Da, np.uint64)
    act_p = ctypes.c_void_p(act_t.ctypes.data)
    a = np.zeros((E, 4, Da), np.float32)
    for i in range(5):
        ref_a = rng.normal(0, 0.5, (E, 4, Da)).astype(np.float32)
        act_t[:] = (np.uint64(i + 1) << np.uint64(32)) | ref_a.reshape(-1).view(np.uint32).astype(np.uint64)
        g = envs[0].step(a, obs_out=obs[0], gate=("tagged", done_p, act_p, ctypes.c_uint32(i + 1), tag_p,
                                                  ctypes.c_uint32(i + 2), ctypes.c_double(1.0)))
        np.testing.assert_array_equal(a, ref_a)
        r = envs[1].step(ref_a, obs_out=obs[1])
        np.testing.assert_array_equal(obs[0], obs[1])
        np.testing.assert_array_equal(g[1], r[1])
        pubs.append(envs[0].published)
        if envs[0].published:
            assert np.all((tagged >> np.uint64(32)) == i + 2)
            np.testing.assert_array_equal((tagged & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32),
                                          obs[0].reshape(-1))
    assert pubs == [True, True, False, True, True]
    gate = lambda: ("tagged", done_p, act_p, ctypes.c_uint32(7), tag_p, ctypes.c_uint32(8), ctypes.c_double(0.05))
    ctr[0] = 0x80000000
    with pytest.raises(RuntimeError, match="observation timed out"):
        envs[0].step(a, obs_out=obs[0], gate=gate())
    ctr[0] = 0
    with pytest.raises(RuntimeError, match="did not finish"):
        envs[0].step(a, obs_out=obs[0], gate=gate())


def test_sampler_stream_bytes_per_geometry():
    """The load-path accounting bench.py divides by the launch time (hopper, bf16, H = 512): the
    streaming kernel ("r") keeps the in/out layers and 2 k-steps of each hidden layer resident
    (loaded once per actor, twice per launch) and streams 14 of 16."""
    code = ("import ctypes, sys; sys.path.insert(0, %r)\n"
            "from diffusionpolicyoptimization_amd import _lib\n"
            "from diffusionpolicyoptimization_amd.ops import ModelDims as Dims\n"
            "d = Dims(obs_dim=11, action_dim=3, horizon_steps=4, cond_steps=1, time_dim=16, actor_hidden=512,"
            " critic_hidden=256, denoising_steps=20, ft_denoising_steps=10)\n"
            "b, w = ctypes.c_int64(), ctypes.c_int()\n"
            "_lib.call('dppo_sampler_stream_bytes', ctypes.byref(d.c()), 1, ctypes.byref(b), ctypes.byref(w))\n"
            "print(b.value, w.value)\n") % ROOT
    got = {}
    for cfg in ("r",):
        out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DPPO_SAMPLER_CFG=cfg),
                             capture_output=True, text=True, check=True).stdout.split()
        got[cfg] = (int(out[0]), int(out[1]))
    assert got["r"] == ((20 * 2 * 14 * 32 + 2 * (64 + 16 + 2 * 2 * 32)) * 1024, 8)


def test_lr_schedules():
    from diffusionpolicyoptimization_amd.util.scheduler import (CosineAnnealingWarmupRestarts,
                                                                CosineAnnealingWarmupRestarts2)
    # shipped cfg: initial = max lr -> constant
    s = CosineAnnealingWarmupRestarts2(1e-4, first_cycle_steps=10, max_lr=1e-4, min_lr=1e-4, warmup_steps=1)
    assert all(abs(s(i) - 1e-4) < 1e-15 for i in range(50))
    s = CosineAnnealingWarmupRestarts2(1e-5, first_cycle_steps=10, max_lr=1e-3, min_lr=1e-5, warmup_steps=2)
    assert s(0) == pytest.approx(1e-5)
    assert s(1) == pytest.approx(1e-5 + (1e-3 - 1e-5) / 2)
    assert s(2) == pytest.approx(1e-3)
    assert s(6) == pytest.approx(1e-5 + (1e-3 - 1e-5) * (1 + math.cos(math.pi * 0.5)) / 2)
    assert s(12) == pytest.approx(1e-3)  # restart: step 12 = step 2 of cycle 1
    e = CosineAnnealingWarmupRestarts(first_cycle_steps=8, max_lr=1.0, min_lr=0.0, warmup_steps=0)
    assert e(0) == pytest.approx(1.0) and e(4) == pytest.approx(0.5) and e(8) == pytest.approx(1.0)

"""The host env boundary: the reference's MultiStep +
MujocoLocomotionLowdimWrapper stack batched in C (csrc/envwrap.c, env/lowdim.py) against a
per-env NumPy restatement of the reference's wrapper code (oracle/envstack.py).

  * the wrapper arithmetic (mujoco_locomotion_lowdim.py:57-62) on the reference's own
    normalization.npz (tests/golden/hopper_medium_v2_normalization.npz): bit-exact;
  * MultiStep (multi_step.py:113-192): reward sums, termination / truncation (incl. a truncation
    in the middle of a chunk and the `cnt += 1` before the `break`), reset within the step and
    final_obs, n_obs_steps stacking with padding, the TimeLimit.truncated branch: bit-exact over
    40 chunks with the C reference simulator and with a Python simulator behind the callbacks;
  * make_async: a gym id without env.synthetic needs MuJoCo and fails loudly; the synthetic
    choices are explicit."""
import os

import numpy as np
import pytest

from oracle.envstack import LinearSimOracle, LowdimWrapperOracle, MultiStepOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NORM = os.path.join(ROOT, "tests", "golden", "hopper_medium_v2_normalization.npz")


def _norm():
    from diffusionpolicyoptimization_amd.env.lowdim import load_normalization
    return load_normalization(NORM)


def test_wrapper_maps_bit_exact_on_reference_normalization():
    from diffusionpolicyoptimization_amd.env import lowdim
    nm = _norm()
    assert nm["obs_min"].shape == (11,) and nm["action_min"].shape == (3,)
    rng = np.random.default_rng(0)
    lo, hi = nm["obs_min"].astype(np.float64), nm["obs_max"].astype(np.float64)
    raw = lo + (hi - lo) * rng.uniform(-0.2, 1.2, (1000, 11))
    orc = LowdimWrapperOracle(None, nm)
    np.testing.assert_array_equal(lowdim.normalize_obs(raw, nm["obs_min"], nm["obs_max"]), orc.normalize_obs(raw))
    a = rng.uniform(-1.5, 1.5, (1000, 3)).astype(np.float32)
    ref = orc.unnormalize_action(a)
    assert ref.dtype == np.float32
    np.testing.assert_array_equal(lowdim.unnormalize_action(a, nm["action_min"], nm["action_max"]), ref)


def _linear_pair(E, seeds, norm, bound_frac):
    from diffusionpolicyoptimization_amd.env.lowdim import LinearSimulator
    sim = LinearSimulator(E, 11, 3, family_seed=3, norm=norm, bound_frac=bound_frac)
    sim.seed(seeds)
    orcs = [LinearSimOracle(sim.A, sim.B, sim.c, sim.goal, sim.center, sim.scale, sim.bound, s) for s in seeds]
    return sim, orcs


def _compare(venv, oracle_envs, E, Ta, n_chunks, rng, amp=1.2):
    obs0 = venv.reset_arg()["state"]
    ref0 = np.stack([o.reset()["state"] for o in oracle_envs]).astype(np.float32)
    np.testing.assert_array_equal(obs0, ref0)
    n_term = n_trunc = n_final = 0
    for _ in range(n_chunks):
        a = rng.uniform(-amp, amp, (E, Ta, venv.action_dim)).astype(np.float32)
        obs, r, term, trunc, infos = venv.step(a)
        for i, o in enumerate(oracle_envs):
            ro, rr, rt, rtr, rinfo = o.step(a[i, :venv.act_steps])
            np.testing.assert_array_equal(obs["state"][i], ro["state"].astype(np.float32))
            assert r[i] == rr and term[i] == rt and trunc[i] == rtr, (i, r[i], rr, term[i], rt, trunc[i], rtr)
            if "final_obs" in rinfo:
                np.testing.assert_array_equal(infos[i]["final_obs"], rinfo["final_obs"]["state"].astype(np.float32))
                n_final += 1
            else:
                assert infos is None or i not in infos
        n_term += int(term.sum())
        n_trunc += int(trunc.sum())
    return n_term, n_trunc, n_final


@pytest.mark.parametrize("To,rws", [(1, True), (2, True), (1, False), (3, True)])
def test_multistep_lowdim_stack_matches_reference_restatement(To, rws):
    from diffusionpolicyoptimization_amd.env.lowdim import LowdimVecEnv
    E, Ta = 7, 4
    nm = _norm()
    seeds = [42 + i for i in range(E)]
    sim, orcs = _linear_pair(E, seeds, nm, bound_frac=0.5)
    venv = LowdimVecEnv(sim, E, 11, 3, act_steps=Ta, n_obs_steps=To, max_episode_steps=10, reset_within_step=rws,
                        normalization=nm)
    oracle_envs = [MultiStepOracle(LowdimWrapperOracle(o, nm), n_obs_steps=To, n_action_steps=Ta,
                                   max_episode_steps=10, reset_within_step=rws) for o in orcs]
    n_term, n_trunc, n_final = _compare(venv, oracle_envs, E, Ta, 40, np.random.default_rng(To))
    assert n_term > 0 and n_trunc > 0, (n_term, n_trunc)        # both ending kinds exercised
    assert (n_final > 0) == rws


class _PySim:
    """A Python simulator reporting TimeLimit.truncated itself (gym's TimeLimit wrapper)."""

    def __init__(self, seed, limit=7):
        self.rng = np.random.default_rng(seed)
        self.limit, self.t, self.s = limit, 0, np.zeros(5)

    def reset(self):
        self.t = 0
        self.s = self.rng.normal(size=5)
        return self.s.copy()

    def step(self, a):
        a = np.asarray(a, np.float64)      # the simulator's control buffer is float64 (mujoco ctrl)
        self.t += 1
        self.s = 0.9 * self.s + 0.1 * np.concatenate([a, a])[:5]
        done = bool(abs(self.s[0]) > 1.2)
        info = {}
        if self.t >= self.limit:
            info["TimeLimit.truncated"] = not done
            done = True
        return self.s.copy(), float(self.s.sum()), done, info


def test_multistep_timelimit_branch_through_python_callbacks():
    from diffusionpolicyoptimization_amd.env.lowdim import CallbackSimulator, LowdimVecEnv
    E, Ta = 5, 4
    sims = [_PySim(10 + i) for i in range(E)]
    orcs = [_PySim(10 + i) for i in range(E)]

    def step(idx, act):
        outs = [sims[i].step(act[r]) for r, i in enumerate(idx)]
        tl = [(-1 if "TimeLimit.truncated" not in o[3] else int(o[3]["TimeLimit.truncated"])) for o in outs]
        return np.stack([o[0] for o in outs]), [o[1] for o in outs], [o[2] for o in outs], tl

    def reset(idx):
        return np.stack([sims[i].reset() for i in idx])

    norm = {"obs_min": -np.ones(5, np.float32), "obs_max": np.ones(5, np.float32),
            "action_min": -2 * np.ones(3, np.float32), "action_max": 2 * np.ones(3, np.float32)}
    venv = LowdimVecEnv(CallbackSimulator(5, 3, step, reset), E, 5, 3, act_steps=Ta, n_obs_steps=2,
                        max_episode_steps=1000, reset_within_step=True, normalization=norm)
    oracle_envs = [MultiStepOracle(LowdimWrapperOracle(o, norm), n_obs_steps=2, n_action_steps=Ta,
                                   max_episode_steps=1000, reset_within_step=True) for o in orcs]
    n_term, n_trunc, _ = _compare(venv, oracle_envs, E, Ta, 25, np.random.default_rng(5))
    assert n_trunc > 0 and n_term > 0


class _GlobalRngEnv:
    """A gym-API env (seed / reset / step -> (obs, reward, done, info)) that draws its noise from the
    process-global NumPy RNG, as the reference's wrapper seeds it (one process per env:
    wrapper/mujoco_locomotion_lowdim.py:39-43); rs: its own RandomState instead (the oracle's
    one-process-per-env stream)."""

    def __init__(self, rs=None, limit=6):
        self.rs, self.limit, self.t, self.s = rs, limit, 0, np.zeros(5)

    def _r(self):
        return self.rs if self.rs is not None else np.random

    def seed(self, s):
        self.seeded = s

    def reset(self):
        self.t = 0
        self.s = 0.5 * self._r().normal(size=5)
        return self.s.copy()

    def step(self, a):
        a = np.asarray(a, np.float64)
        self.t += 1
        self.s = 0.9 * self.s + 0.1 * np.concatenate([a, a])[:5] + 0.05 * self._r().normal(size=5)
        done = bool(abs(self.s[0]) > 1.0)
        info = {}
        if self.t >= self.limit:
            info["TimeLimit.truncated"] = not done
            done = True
        return self.s.copy(), float(self.s.sum()), done, info


def test_gym_simulator_keeps_one_global_rng_stream_per_env(monkeypatch):
    """GymSimulator (env/lowdim.py) over stand-in gym / d4rl modules (the real ones need MuJoCo):
    envs that draw from the global NumPy RNG step through the callback table and the batched
    wrapper stack exactly like one process per env seeded with np.random.seed(seed_i) — each env's
    global-RNG state is swapped in around its calls — and the caller's own global RNG state is left
    untouched."""
    import sys
    import types

    from diffusionpolicyoptimization_amd.env.lowdim import GymSimulator, LowdimVecEnv
    made = []
    gym = types.ModuleType("gym")
    gym.make = lambda env_id: made.append(env_id) or _GlobalRngEnv()
    d4rl = types.ModuleType("d4rl")
    d4rl.gym_mujoco = types.ModuleType("d4rl.gym_mujoco")
    monkeypatch.setitem(sys.modules, "gym", gym)
    monkeypatch.setitem(sys.modules, "d4rl", d4rl)
    monkeypatch.setitem(sys.modules, "d4rl.gym_mujoco", d4rl.gym_mujoco)
    E, Ta = 4, 4
    seeds = [7 + 3 * i for i in range(E)]
    sim = GymSimulator("hopper-medium-v2", E, 5, 3)
    assert made == ["hopper-medium-v2"] * E
    sim.seed(seeds)
    assert [e.seeded for e in sim.envs] == seeds
    norm = {"obs_min": -2 * np.ones(5, np.float32), "obs_max": 2 * np.ones(5, np.float32),
            "action_min": -np.ones(3, np.float32), "action_max": np.ones(3, np.float32)}
    venv = LowdimVecEnv(sim, E, 5, 3, act_steps=Ta, n_obs_steps=1, max_episode_steps=1000,
                        reset_within_step=True, normalization=norm)
    oracle_envs = [MultiStepOracle(LowdimWrapperOracle(_GlobalRngEnv(np.random.RandomState(s)), norm), n_obs_steps=1,
                                   n_action_steps=Ta, max_episode_steps=1000, reset_within_step=True)
                   for s in seeds]
    np.random.seed(12345)
    outer = np.random.get_state()
    n_term, n_trunc, _ = _compare(venv, oracle_envs, E, Ta, 12, np.random.default_rng(3))
    after = np.random.get_state()
    assert after[0] == outer[0] and np.array_equal(after[1], outer[1]) and after[2:] == outer[2:]
    assert n_term + n_trunc > 0


def test_callback_errors_surface():
    from diffusionpolicyoptimization_amd.env.lowdim import CallbackSimulator, LowdimVecEnv

    def step(idx, act):
        raise ValueError("simulator exploded")

    venv = LowdimVecEnv(CallbackSimulator(2, 1, step, lambda idx: np.zeros((len(idx), 2))), 3, 2, 1)
    venv.reset_arg()
    with pytest.raises(RuntimeError, match="simulator exploded"):
        venv.step(np.zeros((3, 4, 1), np.float32))


def test_make_async_is_explicit_about_the_stepper(tmp_path):
    from diffusionpolicyoptimization_amd.env.gym_utils import make_async
    from diffusionpolicyoptimization_amd.env.lowdim import LowdimVecEnv
    from diffusionpolicyoptimization_amd.env.synthetic import SyntheticLocomotionVecEnv
    wr = {"mujoco_locomotion_lowdim": {"normalization_path": NORM},
          "multi_step": {"n_obs_steps": 1, "n_action_steps": 4, "max_episode_steps": 1000, "reset_within_step": True}}
    with pytest.raises(RuntimeError, match="MuJoCo"):
        make_async("hopper-medium-v2", num_envs=2, wrappers=wr, obs_dim=11, action_dim=3)
    with pytest.raises(FileNotFoundError):
        make_async("hopper-medium-v2", num_envs=2, obs_dim=11, action_dim=3,
                   wrappers={"mujoco_locomotion_lowdim": {"normalization_path": str(tmp_path / "missing.npz")}})
    assert isinstance(make_async("hopper-medium-v2", num_envs=2, wrappers=wr, obs_dim=11, action_dim=3,
                                 synthetic=True), SyntheticLocomotionVecEnv)
    v = make_async("hopper-medium-v2", num_envs=2, wrappers=wr, obs_dim=11, action_dim=3, synthetic="lowdim")
    assert isinstance(v, LowdimVecEnv) and v.norm is not None
    o = v.reset_arg()["state"]
    assert o.shape == (2, 1, 11) and np.isfinite(o).all()
    with pytest.raises(ValueError):
        make_async("hopper-medium-v2", num_envs=2, obs_dim=11, action_dim=3, synthetic="mujoco")


# ---- the thread pool and the gated (pipelined) step (csrc/envwrap.c, dppo_lowdim_set_threads) ----
def _lowdim(E, threads, To=2, cost_us=0.0, max_steps=10):
    from diffusionpolicyoptimization_amd.env.lowdim import LinearSimulator, LowdimVecEnv
    nm = _norm()
    sim = LinearSimulator(E, 11, 3, family_seed=3, norm=nm, bound_frac=0.5, cost_us=cost_us)
    sim.seed([42 + i for i in range(E)])
    return LowdimVecEnv(sim, E, 11, 3, act_steps=4, n_obs_steps=To, max_episode_steps=max_steps,
                        reset_within_step=True, normalization=nm, num_threads=threads)


@pytest.mark.parametrize("threads", [2, 3, 8, 64])
def test_thread_pool_is_bit_identical_to_one_thread(threads):
    E = 37                                  # ragged slices
    one, many = _lowdim(E, 1), _lowdim(E, threads)
    many.set_solo_floor(0.0)                # every chunk through the pool
    assert one.num_threads == 1 and many.num_threads == min(threads, E)
    np.testing.assert_array_equal(one.reset_arg()["state"], many.reset_arg()["state"])
    rng = np.random.default_rng(7)
    n_done = 0
    for _ in range(60):
        a = rng.uniform(-1.2, 1.2, (E, 4, 3)).astype(np.float32)
        o1, r1, t1, u1, i1 = one.step(a)
        o2, r2, t2, u2, i2 = many.step(a)
        np.testing.assert_array_equal(o1["state"], o2["state"])
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(t1, t2)
        np.testing.assert_array_equal(u1, u2)
        assert (i1 or {}).keys() == (i2 or {}).keys()
        for k in i1 or {}:
            np.testing.assert_array_equal(i1[k]["final_obs"], i2[k]["final_obs"])
        n_done += int((t1 | u1).sum())
    np.testing.assert_array_equal(one.counters, many.counters)
    assert n_done > 0


def test_thread_pool_survives_resize_and_idle_sleep():
    import time
    v = _lowdim(16, 4)
    v.set_threads(4, spin_us=50.0)          # idle workers sleep after 50 us
    v.reset_arg()
    a = np.zeros((16, 4, 3), np.float32)
    v.step(a)
    time.sleep(0.05)                        # every worker is asleep on the condition variable now
    v.step(a)
    assert v.set_threads(2) == 2 and v.set_threads(1) == 1 and v.set_threads(5) == 5
    v.step(a)
    v.close()


@pytest.mark.parametrize("cost_us,solo", [(0.0, True), (30.0, False)])
def test_solo_floor_steps_cheap_chunks_on_the_caller(cost_us, solo):
    """A trivial simulator's chunk (a few us of work for 16 envs) is below the floor and runs on the
    caller's thread alone; at 30 us per env sub-step (~2 ms per chunk) the pool is used. Outputs match
    a pool that never goes solo, bit for bit."""
    E = 16
    auto, pool = _lowdim(E, 4, cost_us=cost_us), _lowdim(E, 4, cost_us=cost_us)
    auto.set_solo_floor(200.0)              # far from both workloads: robust to a loaded host
    pool.set_solo_floor(0.0)
    np.testing.assert_array_equal(auto.reset_arg()["state"], pool.reset_arg()["state"])
    rng = np.random.default_rng(3)
    for _ in range(30):
        a = rng.uniform(-1.2, 1.2, (E, 4, 3)).astype(np.float32)
        o1, r1, t1, u1, _ = auto.step(a)
        o2, r2, t2, u2, _ = pool.step(a)
        np.testing.assert_array_equal(o1["state"], o2["state"])
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(t1 | u1, t2 | u2)
    assert pool.solo_chunks == 0
    assert (auto.solo_chunks >= 20) if solo else (auto.solo_chunks == 0)
    with pytest.raises(ValueError):
        auto.set_solo_floor(-1.0)


def test_python_simulator_refuses_threads():
    from diffusionpolicyoptimization_amd.env.lowdim import CallbackSimulator, LowdimVecEnv
    sim = CallbackSimulator(2, 1, lambda i, a: None, lambda idx: np.zeros((len(idx), 2)))
    v = LowdimVecEnv(sim, 8, 2, 1)
    assert v.num_threads == 1
    with pytest.raises(ValueError, match="thread-safe"):
        v.set_threads(4)


class _Granules:
    """The mapped-memory side of ops.RolloutPipe's tagged protocol, in plain host memory: the
    device's done word, its action granules {tag : 32, fp32 bits : 32} and the observation
    granules the host publishes."""

    def __init__(self, E, xd, od):
        self.done = np.zeros(16, np.uint32)
        self.act = np.zeros(E * xd, np.uint64)
        self.obs = np.zeros(E * od, np.uint64)

    def put_actions(self, a, tag):
        self.act[:] = (np.uint64(tag) << np.uint64(32)) | a.reshape(-1).view(np.uint32).astype(np.uint64)

    def gate(self, act_tag, obs_tag, timeout=5.0, publish=True):
        import ctypes
        P = lambda x: ctypes.c_void_p(x.ctypes.data)
        return ("tagged", P(self.done), P(self.act), ctypes.c_uint32(act_tag), P(self.obs) if publish else None,
                ctypes.c_uint32(obs_tag), ctypes.c_double(timeout))


@pytest.mark.parametrize("threads", [1, 4])
def test_gated_tagged_step_matches_plain_step(threads):
    """dppo_lowdim_step_gated_tagged: decode the action granules into the caller's buffer, step,
    publish every observation granule with the tag — the same chunk as the plain step."""
    import threading
    import time
    E, To = 24, 2
    ref, gated = _lowdim(E, 1, To=To), _lowdim(E, threads, To=To)
    np.testing.assert_array_equal(ref.reset_arg()["state"], gated.reset_arg()["state"])
    g = _Granules(E, 12, To * 11)
    act_buf = np.zeros((E, 4, 3), np.float32)
    obs_buf = np.zeros((E, To, 11), np.float32)
    rng = np.random.default_rng(3)
    for step in range(1, 31):
        a = rng.uniform(-1.2, 1.2, (E, 4, 3)).astype(np.float32)
        if step % 3 == 0:   # the "device" stores its actions while the slices already spin
            t = threading.Timer(0.002, g.put_actions, (a, step))
            t.start()
        else:
            g.put_actions(a, step)
        o2, r2, t2, u2, _ = gated.step(act_buf, obs_out=obs_buf, gate=g.gate(step, 100 + step))
        if step % 3 == 0:
            t.join()
        assert gated.published
        np.testing.assert_array_equal(act_buf, a)
        o1, r1, t1, u1, _ = ref.step(a)
        np.testing.assert_array_equal(o1["state"], obs_buf)
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(t1 | u1, t2 | u2)
        assert ((g.obs >> np.uint64(32)) == 100 + step).all()
        np.testing.assert_array_equal((g.obs & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                                      obs_buf.reshape(-1).view(np.uint32))
    time.sleep(0)


def test_gated_step_timeouts_and_device_flag():
    E = 8
    v = _lowdim(E, 2)
    v.reset_arg()
    g = _Granules(E, 12, 22)
    act_buf = np.zeros((E, 4, 3), np.float32)
    g.put_actions(act_buf, 1)
    with pytest.raises(RuntimeError, match="did not finish"):
        v.step(act_buf, obs_out=np.zeros((E, 2, 11), np.float32), gate=g.gate(2, 5, timeout=0.05))
    g.done[0] = np.uint32(0x80000000)
    with pytest.raises(RuntimeError, match="device's wait"):
        v.step(act_buf, obs_out=np.zeros((E, 2, 11), np.float32), gate=g.gate(2, 5, timeout=5.0))
    g.done[0] = 0
    with pytest.raises(ValueError, match="C-contiguous"):
        v.step(act_buf[:, :2], gate=g.gate(1, 5))

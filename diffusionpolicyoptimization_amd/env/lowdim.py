"""The reference's gym locomotion env stack on a batched simulator (csrc/envwrap.c):

    AsyncVectorEnv (env/gym_utils/async_vector_env.py:356-456, one worker process per env)
      -> MultiStep (wrapper/multi_step.py:113-192: act_steps sub-steps, reward sum, termination /
         truncation at max_episode_steps, reset within the step, n_obs_steps stacking)
        -> MujocoLocomotionLowdimWrapper (wrapper/mujoco_locomotion_lowdim.py:57-70: obs normalised to
           [-1, 1] by normalization.npz, actions unnormalised)
          -> the simulator

Here the whole stack for all envs is one C call per action chunk (dppo_lowdim_step) that drives a
simulator through a callback table: one batched `step` call per sub-step for the envs still
running, one batched `reset` for the envs whose chunk ended. A simulator is any object with
`step_fn`, `reset_fn` (C function pointers of the dppo_sim types in csrc/envwrap.c) and `ctx`:

  * LinearSimulator — a C simulator (seeded linear dynamics in raw coordinates with a terminal set)
    that fills the table exactly as a MuJoCo C-API stepper would (mj_step per env, the task's
    reward and termination); it runs the stack end to end on hosts without MuJoCo;
  * CallbackSimulator — Python step / reset functions behind ctypes callbacks (test doubles, or a
    simulator with only a Python API);
  * GymSimulator — the reference's own simulator, gym + d4rl + mujoco_py envs, one per env, behind
    a CallbackSimulator (needs those packages: absent on the MI355X hosts).

The wire format is the reference's: reset_arg() -> {"state": [E, To, Do]}; step(actions [E, Ta, Da])
-> ({"state": [E, To, Do]}, reward [E], terminated [E], truncated [E], infos).

Parallelism: the reference runs one worker process per env (async_vector_env.py:189-214). Here the
envs are split into contiguous slices over a pool of host threads inside the C library
(dppo_lowdim_set_threads; `num_threads`, default from the simulator's `thread_safe` flag and the
env count). A C simulator with per-env state (LinearSimulator, a MuJoCo C-API stepper with one
mjData per env) steps its slices concurrently; a Python simulator holds the GIL in every callback,
so it gets one thread unless it says otherwise. Outputs are bit-identical for any thread count.
Below a per-chunk work floor (measured, 25 us by default: `solo_floor_us`, DPPO_ENV_SOLO_FLOOR_US)
a pool steps the chunk on the caller's thread alone, where the hand-off would cost more than the
parallel slices save (a trivial C simulator).

Pipelined rollout: step(..., gate=("tagged", ...)) is the gated host step of ops.RolloutPipe over
this stack (dppo_lowdim_step_gated_tagged): each slice thread polls its envs' action granules,
steps them and publishes their observation granules, so the agent's next sampler launch overlaps
the env step exactly as with the synthetic stepper."""
import ctypes
import os

import numpy as np

from .synthetic import _ENV_LIB

_lib = None
_P = ctypes.c_void_p
STEP_FN = ctypes.CFUNCTYPE(ctypes.c_int, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P)
RESET_FN = ctypes.CFUNCTYPE(ctypes.c_int, _P, ctypes.c_int, _P, _P)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(_ENV_LIB)
        L.dppo_lowdim_create.restype = _P
        L.dppo_lowdim_create.argtypes = [ctypes.c_int] * 7 + [_P, _P, _P, _P, _P, _P, _P]
        L.dppo_lowdim_destroy.argtypes = [_P]
        L.dppo_lowdim_reset_all.argtypes = [_P, _P]
        L.dppo_lowdim_reset_one.argtypes = [_P, ctypes.c_int, _P]
        L.dppo_lowdim_step.argtypes = [_P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P]
        # (h, actions, Ta, reward, term, trunc, obs_out, final_obs, has_final, done, act_tagged, act_tag,
        #  obs_tagged, tag, timeout)
        L.dppo_lowdim_step_gated_tagged.argtypes = [_P, _P, ctypes.c_int] + [_P] * 6 + [_P, _P, ctypes.c_uint32, _P,
                                                                                      ctypes.c_uint32, ctypes.c_double]
        # (h, actions, Ta, reward, term, trunc, obs_out, final_obs, has_final, done, done_target, go, go_value, timeout)
        L.dppo_lowdim_step_gated.argtypes = [_P, _P, ctypes.c_int] + [_P] * 6 + [_P, ctypes.c_uint32, _P,
                                                                               ctypes.c_uint32, ctypes.c_double]
        L.dppo_lowdim_set_threads.argtypes = [_P, ctypes.c_int, ctypes.c_double]
        L.dppo_lowdim_threads.argtypes = [_P]
        L.dppo_lowdim_set_solo_floor.argtypes = [_P, ctypes.c_double]
        L.dppo_lowdim_solo_chunks.restype = ctypes.c_int64
        L.dppo_lowdim_solo_chunks.argtypes = [_P]
        L.dppo_lowdim_normalize_obs.argtypes = [ctypes.c_int64, ctypes.c_int, _P, _P, _P, _P]
        L.dppo_lowdim_normalize_obs.restype = None
        L.dppo_lowdim_unnormalize_action.argtypes = [ctypes.c_int64, ctypes.c_int, _P, _P, _P, _P]
        L.dppo_lowdim_unnormalize_action.restype = None
        L.dppo_lowdim_counters.restype = ctypes.POINTER(ctypes.c_int64)
        L.dppo_lowdim_counters.argtypes = [_P]
        L.dppo_sim_linear_create.restype = _P
        L.dppo_sim_linear_create.argtypes = [ctypes.c_int] * 3 + [_P] * 8
        L.dppo_sim_linear_destroy.argtypes = [_P]
        L.dppo_sim_linear_seed.argtypes = [_P, _P]
        L.dppo_sim_linear_seed.restype = None
        L.dppo_sim_linear_set_cost.argtypes = [_P, ctypes.c_double]
        L.dppo_sim_linear_set_cost.restype = None
        L.dppo_sim_linear_step_fn.restype = _P
        L.dppo_sim_linear_reset_fn.restype = _P
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def normalize_obs(raw, obs_min, obs_max):
    """MujocoLocomotionLowdimWrapper.normalize_obs (:57-58) in the native library; raw float64 [..., Do]."""
    raw = np.ascontiguousarray(raw, np.float64)
    mn, mx = (np.ascontiguousarray(x, np.float32) for x in (obs_min, obs_max))
    out = np.empty_like(raw)
    lib().dppo_lowdim_normalize_obs(raw.size // mn.size, mn.size, _p(raw), _p(mn), _p(mx), _p(out))
    return out


def unnormalize_action(a, action_min, action_max):
    """MujocoLocomotionLowdimWrapper.unnormalize_action (:60-62) in the native library; a float32 [..., Da]."""
    a = np.ascontiguousarray(a, np.float32)
    mn, mx = (np.ascontiguousarray(x, np.float32) for x in (action_min, action_max))
    out = np.empty_like(a)
    lib().dppo_lowdim_unnormalize_action(a.size // mn.size, mn.size, _p(a), _p(mn), _p(mx), _p(out))
    return out


def load_normalization(path):
    """normalization.npz (the reference's data/gym/<task>/normalization.npz): obs_min/obs_max [Do],
    action_min/action_max [Da], float32; loaded without pickle."""
    with np.load(path, allow_pickle=False) as f:
        return {k: np.ascontiguousarray(f[k], np.float32) for k in ("obs_min", "obs_max", "action_min", "action_max")}


class LinearSimulator:
    """dppo_sim_linear (csrc/envwrap.c): raw state s' = A s + B a + c, reward 1 - mean((s' - goal)^2)
    - 1e-3 |a|^2, terminal when any |s'_j - center_j| > bound_j; reset = a seeded hash around `center`. Built
    from a family seed (the dynamics) and the normalisation ranges (the raw coordinate box), so its
    raw observations land in the box the normalisation maps to [-1, 1]. Per-env state only, so the
    pool's threads step disjoint env slices concurrently (thread_safe). cost_us > 0 adds that much
    busy work per env sub-step (a stand-in for a physics step's cost when measuring the pool)."""

    thread_safe = True

    def __init__(self, num_envs, obs_dim, action_dim, family_seed=0, norm=None, bound_frac=0.9, cost_us=0.0):
        rng = np.random.default_rng(20_000 + family_seed)
        if norm is not None:
            lo, hi = norm["obs_min"].astype(np.float64), norm["obs_max"].astype(np.float64)
            alo, ahi = norm["action_min"].astype(np.float64), norm["action_max"].astype(np.float64)
        else:
            lo, hi, alo, ahi = -np.ones(obs_dim), np.ones(obs_dim), -np.ones(action_dim), np.ones(action_dim)
        center, half = (lo + hi) / 2, (hi - lo) / 2
        q, _ = np.linalg.qr(rng.normal(size=(obs_dim, obs_dim)))
        A = (0.95 * q) * half[:, None] / half[None, :]     # a rotation in the normalised coordinates
        # s' - center = A (s - center) + B a + c0: a contraction around center driven by the action
        self.A = np.ascontiguousarray(A)
        self.B = np.ascontiguousarray(rng.normal(0, 0.04, (action_dim, obs_dim)) * half[None, :]
                                      / np.maximum((ahi - alo) / 2, 1e-6)[:, None])
        c0 = rng.normal(0, 0.02, obs_dim) * half
        self.c = np.ascontiguousarray(center - A @ center + c0 - self.B.T @ ((alo + ahi) / 2))
        self.goal = np.ascontiguousarray(center + rng.uniform(-0.3, 0.3, obs_dim) * half)
        self.center, self.scale = np.ascontiguousarray(center), np.ascontiguousarray(0.1 * half)
        # terminal set: leaving the box center +- bound_frac * half (like hopper's healthy-range check)
        self.bound = np.ascontiguousarray(bound_frac * half)
        self.num_envs, self.obs_dim, self.action_dim = num_envs, obs_dim, action_dim
        L = lib()
        seeds = np.arange(num_envs, dtype=np.int64)
        self.ctx = L.dppo_sim_linear_create(num_envs, obs_dim, action_dim, _p(self.A), _p(self.B), _p(self.c),
                                            _p(self.goal), _p(self.center), _p(self.scale), _p(self.bound), _p(seeds))
        if not self.ctx:
            raise MemoryError("dppo_sim_linear_create failed")
        self.step_fn = L.dppo_sim_linear_step_fn()
        self.reset_fn = L.dppo_sim_linear_reset_fn()
        self.set_cost(cost_us)

    def suggested_threads(self, num_envs):
        """Pool size for this simulator: a step of the bare linear dynamics is ~0.1 us per env, below
        the pool's hand-off cost (one thread); with emulated physics work, one thread per 16 envs, at
        most 8."""
        return 1 if self.cost_us < 1.0 else min(8, max(1, num_envs // 16))

    def set_cost(self, cost_us):
        self.cost_us = float(cost_us)
        lib().dppo_sim_linear_set_cost(self.ctx, self.cost_us)

    def seed(self, seeds):
        s = np.ascontiguousarray(np.asarray(list(seeds), np.int64))
        assert s.size == self.num_envs
        lib().dppo_sim_linear_seed(self.ctx, _p(s))

    def __del__(self):
        if getattr(self, "ctx", None) and _lib is not None:
            _lib.dppo_sim_linear_destroy(self.ctx)
            self.ctx = None


class CallbackSimulator:
    """Python simulator behind the callback table. step(idx [n], act [n, Da] f64) -> (obs [n, Do],
    reward [n], done [n] bool, time_limit [n] int: -1 absent, else 0 / 1); reset(idx) -> obs [n, Do].
    The callbacks take the GIL, so the pool steps a Python simulator on one thread unless the
    caller passes thread_safe=True (its step / reset keep per-env state only) and asks for more."""

    def __init__(self, obs_dim, action_dim, step, reset, seed=None, thread_safe=False):
        self.thread_safe = bool(thread_safe)
        self.obs_dim, self.action_dim = obs_dim, action_dim
        self._step, self._reset, self._seed = step, reset, seed
        self.ctx = None
        self.error = None

        def c_step(ctx, n, idx, act, obs, rew, done, tl):
            try:
                ix = np.ctypeslib.as_array(ctypes.cast(idx, ctypes.POINTER(ctypes.c_int32)), (n,)).copy()
                a = np.ctypeslib.as_array(ctypes.cast(act, ctypes.POINTER(ctypes.c_double)), (n, action_dim)).copy()
                o, r, d, t = self._step(ix, a)
                np.ctypeslib.as_array(ctypes.cast(obs, ctypes.POINTER(ctypes.c_double)), (n, obs_dim))[:] = o
                np.ctypeslib.as_array(ctypes.cast(rew, ctypes.POINTER(ctypes.c_double)), (n,))[:] = r
                np.ctypeslib.as_array(ctypes.cast(done, ctypes.POINTER(ctypes.c_uint8)), (n,))[:] = d
                np.ctypeslib.as_array(ctypes.cast(tl, ctypes.POINTER(ctypes.c_int8)), (n,))[:] = t
                return 0
            except Exception as exc:   # reported by LowdimVecEnv.step, never across the C frame
                self.error = exc
                return 1

        def c_reset(ctx, n, idx, obs):
            try:
                ix = np.ctypeslib.as_array(ctypes.cast(idx, ctypes.POINTER(ctypes.c_int32)), (n,)).copy()
                np.ctypeslib.as_array(ctypes.cast(obs, ctypes.POINTER(ctypes.c_double)), (n, obs_dim))[:] = self._reset(ix)
                return 0
            except Exception as exc:
                self.error = exc
                return 1

        self._c_step, self._c_reset = STEP_FN(c_step), RESET_FN(c_reset)   # kept alive with the object
        self.step_fn = ctypes.cast(self._c_step, _P).value
        self.reset_fn = ctypes.cast(self._c_reset, _P).value

    def seed(self, seeds):
        if self._seed is not None:
            self._seed(list(seeds))


class GymSimulator(CallbackSimulator):
    """The reference's simulator: gym.make(id) per env with d4rl's locomotion registrations
    (env/gym_utils/__init__.py:125-174), stepped through the callback table. Needs gym, d4rl and
    mujoco_py; raises ImportError when they are missing (they are absent on the MI355X hosts, so
    it has not run against MuJoCo: its callback and per-env RNG logic runs in
    tests/test_envstack_cpu.py over stand-in gym / d4rl modules). mujoco_py's step holds the
    GIL, so these envs step serially on one thread; a MuJoCo C-API simulator filling the same
    callback table (one mjData per env) is the intended multi-threaded filler.

    RNG: the reference seeds the GLOBAL NumPy RNG of each worker process
    (wrapper/mujoco_locomotion_lowdim.py:39-43), one process per env. In one process a loop of
    np.random.seed calls would leave only the last env's seed, so each env keeps its own global-RNG
    state: it is swapped in around that env's step / reset and saved after, which reproduces the
    per-process streams."""

    def __init__(self, env_id, num_envs, obs_dim, action_dim):
        import gym
        import d4rl.gym_mujoco  # noqa: F401  (registers the *-medium-v2 ids, as the reference does)
        self.envs = [gym.make(env_id) for _ in range(num_envs)]
        self._rng_states = [np.random.get_state() for _ in range(num_envs)]

        def on_env(i, fn):
            outer = np.random.get_state()
            np.random.set_state(self._rng_states[i])
            try:
                return fn(self.envs[i])
            finally:
                self._rng_states[i] = np.random.get_state()
                np.random.set_state(outer)

        def step(idx, act):
            obs = np.empty((len(idx), obs_dim))
            rew, done, tl = np.empty(len(idx)), np.empty(len(idx), bool), np.empty(len(idx), np.int8)
            for r, i in enumerate(idx):
                o, rw, d, info = on_env(i, lambda e: e.step(act[r]))
                obs[r], rew[r], done[r] = o, rw, d
                tl[r] = -1 if "TimeLimit.truncated" not in info else int(bool(info["TimeLimit.truncated"]))
            return obs, rew, done, tl

        def reset(idx):
            return np.stack([np.asarray(on_env(i, lambda e: e.reset()), np.float64) for i in idx])

        def seed(seeds):
            # MujocoLocomotionLowdimWrapper.seed (:39-43): np.random.seed(seed) in the env's own
            # process, plus the simulator's RNG so resets are reproducible
            for i, s in enumerate(seeds):
                outer = np.random.get_state()
                np.random.seed(int(s))
                self._rng_states[i] = np.random.get_state()
                np.random.set_state(outer)
                self.envs[i].seed(int(s))

        super().__init__(obs_dim, action_dim, step, reset, seed)


class LowdimVecEnv:
    """The vector env over a batched simulator (see the module docstring). num_threads: host
    threads that step the envs (None: DPPO_ENV_THREADS, else the simulator's suggested_threads(E),
    else 1)."""

    _PUBLISHED = 1 << 30

    def __init__(self, sim, num_envs, obs_dim, action_dim, act_steps=4, n_obs_steps=1, max_episode_steps=1000,
                 reset_within_step=True, normalization=None, num_threads=None):
        self.sim, self.num_envs, self.obs_dim, self.action_dim = sim, num_envs, obs_dim, action_dim
        self.act_steps, self.n_obs_steps = act_steps, n_obs_steps
        self.max_episode_steps = max_episode_steps
        self.norm = normalization
        self._h = None
        self._make(reset_within_step)
        self.native = lib()            # the agent's gated (pipelined) step runs through this library
        if num_threads is None:
            env_t = os.environ.get("DPPO_ENV_THREADS")
            if env_t:
                num_threads = int(env_t)
            else:
                num_threads = sim.suggested_threads(num_envs) if hasattr(sim, "suggested_threads") else 1
        self.set_threads(num_threads)
        floor = os.environ.get("DPPO_ENV_SOLO_FLOOR_US")
        if floor is not None:
            self.set_solo_floor(float(floor))
        E, To, Do = num_envs, n_obs_steps, obs_dim
        self._reward = np.empty(E)
        self._term = np.empty(E, np.uint8)
        self._trunc = np.empty(E, np.uint8)
        self._final = np.empty((E, To, Do), np.float32)
        self._has_final = np.empty(E, np.uint8)
        self._tail = [_p(x) for x in (self._reward, self._term, self._trunc)]
        self._fin = [_p(self._final), _p(self._has_final)]
        self.published = False

    def set_threads(self, n, spin_us=2000.0):
        """Host threads stepping the envs (the caller's included); returns the count in use."""
        if int(n) > 1 and not getattr(self.sim, "thread_safe", False):
            raise ValueError(f"{type(self.sim).__name__} is not thread-safe: it steps on one thread")
        got = lib().dppo_lowdim_set_threads(self._h, int(n), float(spin_us))
        if got < 1:
            raise RuntimeError("dppo_lowdim_set_threads failed")
        self.num_threads = got
        return got

    def set_solo_floor(self, floor_us):
        """Chunks whose measured stepping work is below floor_us run on the caller's thread alone
        (0: always the pool); see include/dppo_env.h."""
        if lib().dppo_lowdim_set_solo_floor(self._h, float(floor_us)) != 0:
            raise ValueError(f"solo floor {floor_us} us")

    @property
    def solo_chunks(self):
        """Chunks stepped on the caller's thread alone under the solo floor."""
        return int(lib().dppo_lowdim_solo_chunks(self._h))

    def _make(self, reset_within_step):
        L = lib()
        nm = self.norm
        ptrs = [None] * 4 if nm is None else [_p(nm[k]) for k in ("obs_min", "obs_max", "action_min", "action_max")]
        if nm is not None:
            assert nm["obs_min"].size == self.obs_dim and nm["action_min"].size == self.action_dim, "normalization dims"
        self._h = L.dppo_lowdim_create(self.num_envs, self.obs_dim, self.action_dim, self.n_obs_steps, self.act_steps,
                                       int(self.max_episode_steps or 0), int(bool(reset_within_step)),
                                       self.sim.step_fn, self.sim.reset_fn, self.sim.ctx, *ptrs)
        if not self._h:
            raise ValueError("dppo_lowdim_create rejected the env shape")

    def _check(self, rc, what):
        if rc < 0:
            err = getattr(self.sim, "error", None)
            raise RuntimeError(f"simulator {what} failed" + (f": {err!r}" if err is not None else "")) from err

    # ---- reference VectorEnv API ----
    def seed(self, seeds):
        self.sim.seed(seeds)

    def reset_arg(self, options_list=None):
        out = np.empty((self.num_envs, self.n_obs_steps, self.obs_dim), np.float32)
        self._check(lib().dppo_lowdim_reset_all(self._h, _p(out)), "reset")
        return {"state": out}

    def reset_one_arg(self, env_ind, options=None):
        out = np.empty((self.num_envs, self.n_obs_steps, self.obs_dim), np.float32)
        self._check(lib().dppo_lowdim_reset_one(self._h, int(env_ind), _p(out)), "reset")
        return {"state": out[env_ind]}

    @property
    def counters(self):
        return np.ctypeslib.as_array(lib().dppo_lowdim_counters(self._h), (self.num_envs,)).copy()

    def step(self, actions, obs_out=None, gate=None):
        """actions [E, Ta, Da] float32; obs_out: optional float32 [E, To, Do] buffer (pinned / mapped
        staging). gate: the pipelined rollout's arguments (ops.RolloutPipe.gate): ("tagged", done,
        act_tagged, act_tag, obs_tagged, obs_tag, timeout) — the slice threads wait for the device's
        action granules, decode them INTO `actions` (so it must be the caller's own C-contiguous
        float32 array), step, and publish the observation granules — or ("go", done, done_target,
        go, go_value, timeout). self.published tells the caller whether the observation went out."""
        E = self.num_envs
        self.published = False
        a = actions if (isinstance(actions, np.ndarray) and actions.dtype == np.float32
                        and actions.flags.c_contiguous) else np.ascontiguousarray(actions, np.float32)
        if gate is not None and a is not actions:
            raise ValueError("gated steps decode the device's actions into `actions`: pass a C-contiguous "
                             "float32 array")
        ta = a.size // (E * self.action_dim)
        out = obs_out if obs_out is not None else np.empty((E, self.n_obs_steps, self.obs_dim), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == E * self.n_obs_steps * self.obs_dim
        L = lib()
        if gate is None:
            rc = L.dppo_lowdim_step(self._h, _p(a), ta, *self._tail, _p(out), *self._fin)
            self._check(rc, "step")
        else:
            fn = L.dppo_lowdim_step_gated_tagged if gate[0] == "tagged" else L.dppo_lowdim_step_gated
            rc = fn(self._h, _p(a), ta, *self._tail, _p(out), *self._fin, *gate[1:])
            if rc == -2:
                raise RuntimeError("pipelined rollout: the device's wait for the observation timed out")
            self._check(rc, "gated step (simulator error or the sampler step did not finish)")
            self.published = bool(rc & self._PUBLISHED)
        infos = None
        if self._has_final.any():
            infos = {int(i): {"final_obs": self._final[i].copy()} for i in np.nonzero(self._has_final)[0]}
        return ({"state": out}, self._reward.copy(), self._term.astype(bool), self._trunc.astype(bool), infos)

    def close(self):
        if self._h:
            lib().dppo_lowdim_destroy(self._h)
            self._h = None

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.dppo_lowdim_destroy(self._h)
            self._h = None

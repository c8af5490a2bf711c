"""Synthetic locomotion vector env with the wire format of the reference's
AsyncVectorEnv + MultiStep + MujocoLocomotionLowdimWrapper stack
(env/gym_utils/async_vector_env.py:387-456, wrapper/multi_step.py:135-192):
  reset_arg(options_list) -> {"state": [E, To, Do]}
  step(actions [E, Ta, Da]) -> ({"state": [E, To, Do]}, reward [E], terminated [E], truncated [E], infos)

MuJoCo/gym/d4rl are not installed on the MI355X hosts, so episodes follow deterministic seeded
linear dynamics clipped to [-1, 1] (the normalised obs range), a smooth reward, and a fixed
episode length (max_episode_steps sub-steps = 250 chunks at 1000/4) with truncation and
reset-within-step exactly like MultiStep(reset_within_step=True). All envs step together in
vectorised NumPy on the host, which stands in for the C MuJoCo step.
"""
import ctypes
import os

import numpy as np

_ENV_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libdppo_env.so")
_lib = None


def _native():
    """The batched C stepper (csrc/envstep.c); None if it was not built (NumPy path is the spec)."""
    global _lib
    if _lib is None and os.path.exists(_ENV_LIB):
        lib = ctypes.CDLL(_ENV_LIB)
        P = ctypes.c_void_p
        lib.dppo_env_step.argtypes = [ctypes.c_int] * 7 + [P] * 11
        lib.dppo_env_step.restype = ctypes.c_int
        lib.dppo_env_step_gated.argtypes = [ctypes.c_int] * 7 + [P] * 11 + [P, ctypes.c_uint32, P, ctypes.c_uint32,
                                                                            ctypes.c_double]
        lib.dppo_env_step_gated.restype = ctypes.c_int
        # (..., done, act_tagged, act_tag, obs_tagged, tag, timeout)
        lib.dppo_env_step_gated_tagged.argtypes = [ctypes.c_int] * 7 + [P] * 11 + [P, P, ctypes.c_uint32, P,
                                                                                   ctypes.c_uint32, ctypes.c_double]
        lib.dppo_env_step_gated_tagged.restype = ctypes.c_int
        lib.dppo_env_publish_tagged.argtypes = [ctypes.c_int64, P, P, ctypes.c_uint32]
        lib.dppo_env_publish_tagged.restype = None
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


class SyntheticLocomotionVecEnv:
    def __init__(self, num_envs, obs_dim, action_dim, act_steps=4, n_obs_steps=1, max_episode_steps=1000,
                 family_seed=0, native=True):
        self.num_envs, self.obs_dim, self.action_dim = num_envs, obs_dim, action_dim
        self.act_steps, self.n_obs_steps, self.max_episode_steps = act_steps, n_obs_steps, max_episode_steps
        rng = np.random.default_rng(10_000 + family_seed)
        q, _ = np.linalg.qr(rng.normal(size=(obs_dim, obs_dim)))
        self.A = (0.97 * q).astype(np.float64)                        # stable rotation-like dynamics
        self.B = rng.normal(0, 0.3, size=(action_dim, obs_dim))
        self.c = rng.normal(0, 0.02, size=obs_dim)
        self.goal = rng.uniform(-0.5, 0.5, size=obs_dim)
        self.native = _native() if native else None
        self._reward = np.empty(num_envs)
        self._term = np.zeros(num_envs, dtype=np.uint8)
        self._trunc = np.zeros(num_envs, dtype=np.uint8)
        self._static_ptrs = None
        self._last_a = self._last_o = None
        self.seeds = np.arange(num_envs)
        self.state = np.zeros((num_envs, obs_dim))
        self.cnt = np.zeros(num_envs, dtype=np.int64)
        self.episode = np.zeros(num_envs, dtype=np.int64)

    # ---- reference VectorEnv API ----
    def seed(self, seeds):
        self.seeds = np.asarray(list(seeds), dtype=np.int64)

    def _initial(self, idx):
        """Seeded initial state of episode `episode[i]` of env i: U(-0.1, 0.1)^Do from a hash of
        (env seed, episode index, coordinate) — deterministic and cheap to vectorise."""
        idx = np.asarray(idx)
        sd = self.seeds[idx].astype(np.float64)[:, None]
        ep = self.episode[idx].astype(np.float64)[:, None]
        j = np.arange(self.obs_dim, dtype=np.float64)[None, :]
        h = np.sin(sd * 12.9898 + ep * 78.233 + j * 37.719 + 0.5) * 43758.5453
        return (h - np.floor(h) - 0.5) * 0.2

    def _obs(self):
        return {"state": np.repeat(self.state[:, None, :], self.n_obs_steps, axis=1).copy()}

    def reset_arg(self, options_list=None):
        idx = np.arange(self.num_envs)
        self.state[:] = self._initial(idx)
        self.cnt[:] = 0
        return self._obs()

    def reset_one_arg(self, env_ind, options=None):
        self.state[env_ind] = self._initial([env_ind])[0]
        self.cnt[env_ind] = 0
        return {"state": np.repeat(self.state[env_ind][None], self.n_obs_steps, axis=0)}

    _PUBLISHED = 1 << 30

    def step(self, actions, obs_out=None, gate=None):
        """actions [E, Ta, Da]; obs_out: optional float32 [E, To, Do] buffer (e.g. pinned staging).
        gate: ("go", done_addr, done_target, go_addr, go_value, timeout) or
        ("tagged", done_addr, act_tagged_addr, act_tag, obs_tagged_addr, obs_tag, timeout) of a pipelined rollout
        (ops.RolloutPipe.gate): the native stepper waits for the device's done counter, steps, and
        publishes the observation itself (go counter, or tagged granules) when no env needs a reset;
        self.published tells the caller whether it did."""
        E = self.num_envs
        self.published = False
        if gate is not None and self.native is None:
            raise RuntimeError("gated env steps need the native stepper (lib/libdppo_env.so)")
        if self.native is not None:
            a = actions if (isinstance(actions, np.ndarray) and actions.dtype == np.float32
                            and actions.flags.c_contiguous) else np.ascontiguousarray(actions, dtype=np.float32)
            if gate is not None and gate[0] == "tagged" and a is not actions:
                # the tagged stepper decodes the device's actions INTO this buffer: it must be the
                # caller's own [E, Ta, Da] array, not a contiguous copy of a strided view
                raise ValueError("tagged gated steps need C-contiguous float32 actions")
            ta = a.size // (E * self.action_dim)
            out = obs_out if obs_out is not None else np.empty((E, self.n_obs_steps, self.obs_dim), np.float32)
            if self._static_ptrs is None:
                self.state = np.ascontiguousarray(self.state)
                self._AT = np.ascontiguousarray(self.A.T)
                self._static_ptrs = [_p(x) for x in (self._AT, self.B, self.c, self.goal, self.state, self.cnt)]
                self._tail_ptrs = [_p(x) for x in (self._reward, self._term, self._trunc)]
            # pointer caches keyed by object identity (the reference held here keeps the id unique)
            if a is not self._last_a:
                self._last_a, self._last_pa = a, _p(a)
            if out is not self._last_o:
                self._last_o, self._last_po = out, _p(out)
            if gate is None:
                n_done = self.native.dppo_env_step(E, self.obs_dim, self.action_dim, self.act_steps, ta,
                                                   self.max_episode_steps, self.n_obs_steps, *self._static_ptrs,
                                                   self._last_pa, *self._tail_ptrs, self._last_po)
            else:
                # gate[0] names the protocol: "go" (counter) or "tagged" (tagged observation granules)
                fn = self.native.dppo_env_step_gated_tagged if gate[0] == "tagged" else self.native.dppo_env_step_gated
                rc = fn(E, self.obs_dim, self.action_dim, self.act_steps, ta, self.max_episode_steps,
                        self.n_obs_steps, *self._static_ptrs, self._last_pa, *self._tail_ptrs, self._last_po, *gate[1:])
                if rc < 0:
                    raise RuntimeError("pipelined rollout: " + ("the device's wait for the observation timed out"
                                                                if rc == -2 else "the sampler step did not finish"))
                self.published = bool(rc & self._PUBLISHED)
                n_done = rc & (self._PUBLISHED - 1)
            reward = self._reward.copy()
            terminated, truncated = self._term.astype(bool), self._trunc.astype(bool)
        else:
            a = np.asarray(actions, np.float64).reshape(E, -1, self.action_dim)[:, :self.act_steps]
            reward = np.zeros(E)
            terminated = np.zeros(E, dtype=bool)
            truncated = np.zeros(E, dtype=bool)
            alive = np.ones(E, dtype=bool)
            for k in range(a.shape[1]):                               # MultiStep.step (multi_step.py:146-170)
                self.cnt[alive] += 1
                s = self.state @ self.A.T + np.clip(a[:, k], -1, 1) @ self.B + self.c
                s = np.clip(s, -1.0, 1.0)
                self.state = np.where(alive[:, None], s, self.state)
                r = 1.0 - np.mean((self.state - self.goal) ** 2, axis=1) - 0.01 * np.mean(a[:, k] ** 2, axis=1)
                reward += np.where(alive, r, 0.0)                     # reward_agg_method = "sum"
                truncated |= alive & (self.cnt >= self.max_episode_steps)
                alive &= ~truncated
            out = None
        infos = None
        if (n_done if self.native is not None else (terminated | truncated).any()):  # reset_within_step
            done = terminated | truncated                                            # (multi_step.py:177-187)
            idx = np.nonzero(done)[0]
            infos = {int(i): {"final_obs": self.state[i].copy()} for i in idx}
            self.episode[idx] += 1
            self.state[idx] = self._initial(idx)
            self.cnt[idx] = 0
            if out is not None:
                out[idx] = self.state[idx, None, :].astype(np.float32)
        obs = {"state": out} if out is not None else self._obs()
        return obs, reward, terminated, truncated, infos

    def close(self):
        pass

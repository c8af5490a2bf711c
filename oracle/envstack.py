"""TEST INFRASTRUCTURE ONLY (tests/ and the CPU baseline may import it; the product never does).

A restatement of the reference's gym locomotion wrapper stack, one env at a time in NumPy, as the
reference writes it:
  * MujocoLocomotionLowdimWrapper — env/gym_utils/wrapper/mujoco_locomotion_lowdim.py:45-70
    (reset / normalize_obs / unnormalize_action / step);
  * MultiStep — env/gym_utils/wrapper/multi_step.py:113-192 (reset, step with the cnt / break
    order, TimeLimit.truncated handling, reward "sum", reset within the step, final_obs) and
    stack_last_n_obs (:68-78);
  * LinearSimOracle — the restatement of the C reference simulator dppo_sim_linear
    (csrc/envwrap.c), element loops in the C code's order so results are bit-identical.

The wrapper arithmetic is pinned by the reference's own data file (normalization.npz, copied to
tests/golden/hopper_medium_v2_normalization.npz) and the reference's dtypes: float32 actions,
float64 simulator observations. gym, d4rl and mujoco_py are not installed, so the simulator under
the wrappers is a stand-in (parity of the simulator itself is out of reach here)."""
from collections import deque

import numpy as np


class LowdimWrapperOracle:
    """mujoco_locomotion_lowdim.py:12-70 over a per-env simulator with step(a) -> (obs, r, done,
    info) and reset() -> obs."""

    def __init__(self, sim, norm):
        self.env = sim
        self.obs_min, self.obs_max = norm["obs_min"], norm["obs_max"]                 # :21-25
        self.action_min, self.action_max = norm["action_min"], norm["action_max"]

    def reset(self):
        return {"state": self.normalize_obs(self.env.reset())}                       # :45-55

    def normalize_obs(self, obs):                                                    # :57-58
        return 2 * ((obs - self.obs_min) / (self.obs_max - self.obs_min + 1e-6) - 0.5)

    def unnormalize_action(self, action):                                            # :60-62
        action = (action + 1) / 2
        return action * (self.action_max - self.action_min) + self.action_min

    def step(self, action):                                                          # :64-70
        raw_action = self.unnormalize_action(action)
        raw_obs, reward, done, info = self.env.step(raw_action)
        return {"state": self.normalize_obs(raw_obs)}, reward, done, info


def stack_last_n_obs(all_obs, n_steps):                                              # multi_step.py:68-78
    all_obs = list(all_obs)
    result = np.zeros((n_steps,) + all_obs[-1].shape, dtype=all_obs[-1].dtype)
    start_idx = -min(n_steps, len(all_obs))
    result[start_idx:] = np.array(all_obs[start_idx:])
    if n_steps > len(all_obs):
        result[:start_idx] = result[start_idx]
    return result


class MultiStepOracle:
    """multi_step.py:81-192 (state observations, prev_action and info deques dropped: they do not
    reach the agent)."""

    def __init__(self, env, n_obs_steps=1, n_action_steps=1, max_episode_steps=None, reset_within_step=False):
        self.env = env
        self.n_obs_steps, self.n_action_steps = n_obs_steps, n_action_steps
        self.max_episode_steps, self.reset_within_step = max_episode_steps, reset_within_step

    def reset(self):                                                                 # :113-133
        obs = self.env.reset()
        self.obs = deque([obs], maxlen=max(self.n_obs_steps + 1, self.n_action_steps))
        self.reward, self.done = [], []
        self.cnt = 0
        return self._get_obs(self.n_obs_steps)

    def step(self, action):                                                          # :135-192
        if action.ndim == 1:
            action = action[None]
        truncated = terminated = False
        info = {}
        for act in action:
            self.cnt += 1
            if terminated or truncated:
                break
            observation, reward, done, info = self.env.step(act)
            self.obs.append(observation)
            self.reward.append(reward)
            if "TimeLimit.truncated" not in info:
                if done:
                    terminated = True
                elif self.max_episode_steps is not None and self.cnt >= self.max_episode_steps:
                    truncated = True
            else:
                truncated = info["TimeLimit.truncated"]
                terminated = done
            done = truncated or terminated
            self.done.append(done)
        observation = self._get_obs(self.n_obs_steps)
        reward = np.sum(self.reward)                                                 # aggregate "sum"
        out_info = {}
        if self.reset_within_step and self.done[-1]:
            if truncated:
                out_info["final_obs"] = observation
            observation = self.reset()
        self.reward, self.done = [], []
        return observation, reward, terminated, truncated, out_info

    def _get_obs(self, n_steps):
        return {"state": stack_last_n_obs([o["state"] for o in self.obs], n_steps)}


class LinearSimOracle:
    """dppo_sim_linear for ONE env (csrc/envwrap.c), the C loop order kept."""

    def __init__(self, A, B, c, goal, center, scale, bound, seed):
        self.A, self.B, self.c, self.goal = A, B, c, goal
        self.center, self.scale, self.bound = center, scale, bound
        self.seed, self.episode = int(seed), 0
        self.s = np.zeros(len(c))

    def reset(self):
        M = (1 << 64) - 1
        Do = len(self.c)
        s = np.zeros(Do)
        for j in range(Do):
            z = (self.seed * 0x9E3779B97F4A7C15 + self.episode * 0xBF58476D1CE4E5B9 + j * 0x94D049BB133111EB + 1) & M
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
            z ^= z >> 31
            u = float(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0
            s[j] = self.center[j] + self.scale[j] * u
        self.episode += 1
        self.s = s
        return s.copy()

    def step(self, a):
        a = np.asarray(a, np.float64)
        Do, Da = len(self.c), len(a)
        sn = np.zeros(Do)
        err, asq, out = 0.0, 0.0, False
        for j in range(Do):
            v = float(self.c[j])
            for q in range(Do):
                v += float(self.A[j, q]) * float(self.s[q])
            for q in range(Da):
                v += float(self.B[q, j]) * float(a[q])
            sn[j] = v
            d = v - float(self.goal[j])
            err += d * d
            dc = v - float(self.center[j])
            out |= dc > float(self.bound[j]) or dc < -float(self.bound[j])
        for q in range(Da):
            asq += float(a[q]) * float(a[q])
        self.s = sn
        return sn.copy(), 1.0 - err / Do - 1e-3 * asq, bool(out), {}


class LowdimVecEnvOracle:
    """The vector env of the loop oracle (oracle/iteration.py) over E MultiStep(LowdimWrapper(sim))
    envs (reset_within_step, To = 1): the reference's actions reach the wrapper as float32."""

    def __init__(self, sims, norm, obs_dim, action_dim, act_steps, max_episode_steps):
        self.envs = [MultiStepOracle(LowdimWrapperOracle(s, norm), n_obs_steps=1, n_action_steps=act_steps,
                                     max_episode_steps=max_episode_steps, reset_within_step=True) for s in sims]
        self.E, self.obs_dim, self.action_dim = len(sims), obs_dim, action_dim

    def reset_all(self):
        return np.stack([e.reset()["state"][-1] for e in self.envs])

    def step(self, actions):
        outs = [e.step(np.asarray(actions[i], np.float32)) for i, e in enumerate(self.envs)]
        obs = np.stack([o[0]["state"][-1] for o in outs])
        return (obs, np.array([o[1] for o in outs], np.float64), np.array([o[2] for o in outs], bool),
                np.array([o[3] for o in outs], bool))

"""make_async (reference env/gym_utils/__init__.py:10-231) for the MI355X host.

The reference spawns one gym+MuJoCo worker process per env. gym, d4rl and MuJoCo are not
installed on these hosts, so the gym locomotion ids resolve to the synthetic vector env with
the same wire format (env/synthetic.py) and any other id fails loudly."""
from .synthetic import SyntheticLocomotionVecEnv

_LOCOMOTION = ("hopper", "walker2d", "halfcheetah", "ant", "synthetic")


def make_async(id, num_envs=1, asynchronous=True, wrappers=None, render=False, obs_dim=23, action_dim=7,
               env_type=None, max_episode_steps=None, act_steps=4, obs_steps=1, family_seed=0, native=True, **kwargs):
    name = str(id).lower()
    if env_type not in (None, "gym") or not any(name.startswith(p) for p in _LOCOMOTION):
        raise NotImplementedError(f"env {id!r} (type {env_type}): only the gym locomotion tasks are in scope")
    try:  # a real MuJoCo install would plug in here; none exists on the MI355X pool
        import gym  # noqa: F401
        import mujoco_py  # noqa: F401
        raise NotImplementedError("MuJoCo stepping backend: SURVEY.md §8(f) rank 1 (not built this round)")
    except ImportError:
        pass
    w = wrappers or {}
    ms = w.get("multi_step", {}) if isinstance(w, dict) else {}
    return SyntheticLocomotionVecEnv(num_envs, obs_dim, action_dim,
                                     act_steps=ms.get("n_action_steps", act_steps),
                                     n_obs_steps=ms.get("n_obs_steps", obs_steps),
                                     max_episode_steps=ms.get("max_episode_steps", max_episode_steps or 1000),
                                     family_seed=family_seed, native=native)

"""make_async (reference env/gym_utils/__init__.py:10-231) for the MI355X host.

Which stepper runs is explicit, never a silent substitution:
  * env.synthetic: true (or an id starting with "synthetic") — the synthetic linear env in the
    normalised space (env/synthetic.py), stepped by the AVX2 C stepper with the pipelined
    tagged-granule protocol; the bench workload;
  * env.synthetic: lowdim — the reference's wrapper stack (MultiStep + MujocoLocomotionLowdimWrapper,
    batched in C: env/lowdim.py, csrc/envwrap.c) over the C reference simulator in raw coordinates,
    with the cfg's normalization.npz when the file exists;
  * otherwise (the reference's own cfgs) — the real simulator: gym + d4rl + mujoco_py envs behind the
    same C wrapper stack. Without those packages this fails loudly and says how to choose a
    synthetic env."""
import os

from .lowdim import GymSimulator, LinearSimulator, LowdimVecEnv, load_normalization
from .synthetic import SyntheticLocomotionVecEnv

_LOCOMOTION = ("hopper", "walker2d", "halfcheetah", "ant", "synthetic")


def _wrapper_args(wrappers):
    w = wrappers or {}
    ms = w.get("multi_step", {}) if hasattr(w, "get") else {}
    lo = w.get("mujoco_locomotion_lowdim", {}) if hasattr(w, "get") else {}
    return (ms or {}), (lo or {})


def make_async(id, num_envs=1, asynchronous=True, wrappers=None, render=False, obs_dim=23, action_dim=7,
               env_type=None, max_episode_steps=None, act_steps=4, obs_steps=1, family_seed=0, native=True,
               synthetic=False, num_threads=None, sim_cost_us=0.0, **kwargs):
    """num_threads: host threads stepping the wrapper stack (LowdimVecEnv; None: its default).
    sim_cost_us: emulated work per env sub-step of the C reference simulator (measurement only)."""
    name = str(id).lower()
    if env_type not in (None, "gym") or not any(name.startswith(p) for p in _LOCOMOTION):
        raise NotImplementedError(f"env {id!r} (type {env_type}): only the gym locomotion tasks are in scope")
    ms, lo = _wrapper_args(wrappers)
    n_act = ms.get("n_action_steps", act_steps)
    n_obs = ms.get("n_obs_steps", obs_steps)
    max_steps = ms.get("max_episode_steps", max_episode_steps or 1000)
    rws = bool(ms.get("reset_within_step", True))
    if synthetic is True or name.startswith("synthetic"):
        return SyntheticLocomotionVecEnv(num_envs, obs_dim, action_dim, act_steps=n_act, n_obs_steps=n_obs,
                                         max_episode_steps=max_steps, family_seed=family_seed, native=native)
    npath = lo.get("normalization_path")
    norm = load_normalization(npath) if npath and os.path.exists(str(npath)) else None
    if synthetic == "lowdim":
        sim = LinearSimulator(num_envs, obs_dim, action_dim, family_seed=family_seed, norm=norm, cost_us=sim_cost_us)
        return LowdimVecEnv(sim, num_envs, obs_dim, action_dim, act_steps=n_act, n_obs_steps=n_obs,
                            max_episode_steps=max_steps, reset_within_step=rws, normalization=norm,
                            num_threads=num_threads)
    if synthetic not in (False, None):
        raise ValueError(f"env.synthetic must be true, 'lowdim' or false, got {synthetic!r}")
    # the reference's simulator (env/gym_utils/__init__.py:125-174: d4rl.gym_mujoco + gym.make per env)
    if npath and norm is None:
        raise FileNotFoundError(f"normalization file {npath!r} (wrappers.mujoco_locomotion_lowdim) does not exist")
    try:
        sim = GymSimulator(id, num_envs, obs_dim, action_dim)
    except ImportError as exc:
        raise RuntimeError(
            f"env {id!r} needs the MuJoCo simulator (gym + d4rl + mujoco_py), which is not installed here "
            f"({exc}). Set env.synthetic=true for the synthetic locomotion env with the same wire format "
            "(the bench workload), or env.synthetic=lowdim for the reference's wrapper stack over the C "
            "reference simulator.") from exc
    if "mujoco_locomotion_lowdim" not in (wrappers or {}):
        norm = None
    return LowdimVecEnv(sim, num_envs, obs_dim, action_dim, act_steps=n_act, n_obs_steps=n_obs,
                        max_episode_steps=max_steps, reset_within_step=rws, normalization=norm,
                        num_threads=num_threads)

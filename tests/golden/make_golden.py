"""Generate tests/golden/*.npz from the REFERENCE where it is importable in the build container.

Run from the repo root in the build container (needs /root/reference):
    python tests/golden/make_golden.py
Only util/reward_scaling.py of the reference imports without TensorFlow; it is
imported here, run on seeded inputs, and its outputs are stored as data. Nothing from the
reference is copied; the GPU box only ever sees the .npz files.
"""
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def reward_scaling():
    sys.path.insert(0, REF)
    from util.reward_scaling import RunningRewardScaler  # the reference implementation
    sys.path.pop(0)
    rng = np.random.default_rng(2024)
    cases = {}
    for ci, (E, S, n_calls) in enumerate([(4, 50, 3), (64, 120, 2), (1, 7, 4), (5, 1, 3)]):
        sc = RunningRewardScaler(E)
        for k in range(n_calls):
            r = rng.normal(1.5, 2.5, size=(E, S))
            first = (rng.uniform(size=(E, S)) < 0.03).astype(np.float64)
            if k == 0:
                first[:, 0] = 1.0
            out = sc(reward=r, first=first)
            p = f"c{ci}_k{k}_"
            cases[p + "reward"] = r
            cases[p + "first"] = first
            cases[p + "out"] = out
            cases[p + "rms"] = np.array([sc.ret_rms.mean, sc.ret_rms.var, sc.ret_rms.count])
            cases[p + "ret"] = sc.ret.copy()
        cases[f"c{ci}_meta"] = np.array([E, S, n_calls])
    np.savez_compressed(os.path.join(OUT, "reward_scaling.npz"), **cases)


def reward_scaling_per_env():
    """RunningRewardScaler(per_env=True) (reward_scaling.py:51-66): the state has shape (num_envs,)
    and is updated by moments over axis 0 of rets [E, S] (the envs), joined by NumPy broadcasting.
    Cases the reference runs: S == E; E == 1 (the state takes S's shape); S == 1 (the output
    broadcasts to [E, E]); and one it rejects (E = 4, S = 50: ValueError), stored as a flag."""
    sys.path.insert(0, REF)
    from util.reward_scaling import RunningRewardScaler  # the reference implementation
    sys.path.pop(0)
    rng = np.random.default_rng(2025)
    cases = {}
    plans = [(4, [4, 4, 4]), (16, [16, 16]), (1, [7, 7, 1]), (5, [1, 1]), (3, [3, 1, 3]), (4, [50])]
    for ci, (E, Ss) in enumerate(plans):
        sc = RunningRewardScaler(E, per_env=True)
        for k, S in enumerate(Ss):
            r = rng.normal(1.5, 2.5, size=(E, S))
            first = (rng.uniform(size=(E, S)) < 0.05).astype(np.float64)
            if k == 0:
                first[:, 0] = 1.0
            p = f"c{ci}_k{k}_"
            cases[p + "reward"] = r
            cases[p + "first"] = first
            try:
                out = sc(reward=r, first=first)
            except ValueError:
                cases[p + "raises"] = np.array(1)
                break
            cases[p + "out"] = out
            cases[p + "mean"] = np.asarray(sc.ret_rms.mean)
            cases[p + "var"] = np.asarray(sc.ret_rms.var)
            cases[p + "count"] = np.asarray(sc.ret_rms.count)
            cases[p + "ret"] = sc.ret.copy()
        cases[f"c{ci}_meta"] = np.array([E, len(Ss)])
    np.savez_compressed(os.path.join(OUT, "reward_scaling_per_env.npz"), **cases)


def normalization():
    src = os.path.join(REF, "data/gym/hopper-medium-v2/normalization.npz")
    with np.load(src, allow_pickle=False) as f:
        np.savez(os.path.join(OUT, "hopper_medium_v2_normalization.npz"), **{k: f[k] for k in f.files})


if __name__ == "__main__":
    reward_scaling()
    reward_scaling_per_env()
    normalization()
    print("wrote", sorted(os.listdir(OUT)))

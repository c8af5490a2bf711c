"""Host-side cost of one action chunk of the wrapper stack (csrc/envwrap.c) vs pool threads, on the
C linear simulator with an optional emulated per-env sub-step cost (LinearSimulator cost_us).

    python tools/env_pool_bench.py [--envs 64] [--cost-us 0 20] [--threads 1 2 4 8]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from diffusionpolicyoptimization_amd.env.lowdim import LinearSimulator, LowdimVecEnv, load_normalization
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--cost-us", type=float, nargs="+", default=[0.0, 20.0])
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--chunks", type=int, default=300)
    a = ap.parse_args()
    norm = load_normalization(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "tests", "golden", "hopper_medium_v2_normalization.npz"))
    E = a.envs
    out = []
    for cost in a.cost_us:
        for th in a.threads:
            sim = LinearSimulator(E, 11, 3, norm=norm, cost_us=cost)
            v = LowdimVecEnv(sim, E, 11, 3, act_steps=4, max_episode_steps=1000, normalization=norm, num_threads=th)
            v.reset_arg()
            act = np.zeros((E, 4, 3), np.float32)
            obs = np.zeros((E, 1, 11), np.float32)
            for _ in range(20):
                v.step(act, obs_out=obs)
            n = a.chunks if cost == 0 else max(20, a.chunks // 5)
            t0 = time.perf_counter()
            for _ in range(n):
                v.step(act, obs_out=obs)
            us = (time.perf_counter() - t0) / n * 1e6
            out.append({"envs": E, "cost_us_per_env_substep": cost, "threads": v.num_threads, "us_per_chunk": us})
            print(json.dumps(out[-1]), flush=True)
            v.close()


if __name__ == "__main__":
    main()

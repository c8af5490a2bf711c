"""Where a pipelined rollout step's time goes on the device: runs bench.py's workload (hopper, 64
envs, S=500) for one warm-up iteration, then one rollout with a timing build of the split sampler
(DPPO_LIB=<stime variant>, tools/variant_build.sh stime -DDPPO_SAMPLER_TIMING) and prints the
per-launch average of each kernel phase in shader cycles, plus the host's wall time per step.
    DPPO_LIB=... python tools/rollout_probe.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from diffusionpolicyoptimization_amd import _lib
    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      ["env.n_envs=64", "train.force_train=True", "train.save_checkpoints=False",
                       "train.save_results=False", "logdir=/tmp/dppo_probe"])
    agent = get_class(cfg._target_)(cfg)
    agent.iteration(force_train=True)
    lib = _lib.load()
    timing = hasattr(lib, "dppo_debug_split_cycles")
    buf = (ctypes.c_ulonglong * (16 + 64 * 8))()
    if timing:
        lib.dppo_debug_split_cycles(buf, 1)
    # host side: wall time inside each call of the rollout loop
    pipe, venv = agent.pipe, agent.venv
    acc = {"enqueue": 0.0, "env_step": 0.0}
    orig_enq, orig_step = pipe.enqueue, venv.step

    def enq(*a, **k):
        t = time.perf_counter()
        r = orig_enq(*a, **k)
        acc["enqueue"] += time.perf_counter() - t
        return r

    def step(*a, **k):
        t = time.perf_counter()
        r = orig_step(*a, **k)
        acc["env_step"] += time.perf_counter() - t
        return r
    pipe.enqueue, venv.step = enq, step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.rollout(eval_mode=False)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    pipe.enqueue, venv.step = orig_enq, orig_step
    if timing:
        lib.dppo_debug_split_cycles(buf, 1)
    S = cfg.train.n_steps
    wgs = 8 * ((agent.n_envs + 15) // 16)
    names = {0: "prologue_after_go", 1: "loop_top", 2: "in", 3: "l1", 4: "l2_out", 5: "xchg", 6: "epilogue",
             7: "prologue_before_go", 8: "go_wait", 9: "tail", 10: "done_signal"}
    per = {n: round(buf[k] / wgs / S / (agent.model.dims.denoising_steps if 1 <= k <= 6 else 1))
           for k, n in names.items()}
    host = {k: v / S * 1e6 for k, v in acc.items()}
    print(json.dumps({"rollout_wall_us_per_step": wall / S * 1e6, "host_us_per_step": host,
                      "cycles_per_launch_or_step": per if timing else None}), flush=True)


if __name__ == "__main__":
    main()

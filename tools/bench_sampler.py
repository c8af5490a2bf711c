"""Times the K-step sampler alone on the bench workload (hopper, bf16, 64 envs): back-to-back
launches bracketed by HIP events on the launch stream. Writes the actions of a fixed-seed call
to gpurun_out/sampler_<tag>.npy so variants (DPPO_SAMPLER_QD) can be compared bit for bit.
    python tools/bench_sampler.py [--envs 64] [--reps 200] [--tag qd3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _split(m, envs):
    from diffusionpolicyoptimization_amd import ops
    return ops.sampler_layout(m.dims, m.precision, envs) > 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--tag", default=os.environ.get("DPPO_SAMPLER_QD", "default"))
    args = ap.parse_args()
    import numpy as np
    import torch

    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    dev = torch.device("cuda:0")
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      [f"model.precision={args.precision}"])
    m = instantiate(cfg.model, device=dev, seed=0)
    cond = torch.rand(args.envs, m.dims.sd, device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 2 - 1
    m._call_id = 0
    ref = m(cond).trajectories.cpu().numpy()
    for _ in range(5):
        m(cond)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        m(cond)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"sampler_{args.tag}.npy"), ref)
    d = m.dims
    flops = d.denoising_steps * 2 * (d.actor_in * d.actor_hidden + 2 * d.actor_hidden ** 2 + d.actor_hidden * d.xd) * args.envs
    phases = None
    from diffusionpolicyoptimization_amd import _lib
    lib = _lib.load()
    if hasattr(lib, "dppo_debug_sampler_cycles"):   # timing build: cycles per phase per denoising step
        import ctypes
        buf = (ctypes.c_ulonglong * 16)()
        lib.dppo_debug_sampler_cycles(buf, 1)
        m(cond)
        torch.cuda.synchronize()
        lib.dppo_debug_sampler_cycles(buf, 1)
        wgs = (args.envs + 15) // 16
        phases = {f"s{i}": round(buf[i] / wgs / (d.denoising_steps if i else 1)) for i in range(7)}
    if hasattr(lib, "dppo_debug_split_cycles") and _split(m, args.envs):   # split kernel phases
        import ctypes
        buf = (ctypes.c_ulonglong * (16 + 64 * 8))()
        lib.dppo_debug_split_cycles(buf, 1)
        m(cond)
        torch.cuda.synchronize()
        lib.dppo_debug_split_cycles(buf, 1)
        wgs = 8 * ((args.envs + 15) // 16)
        names = ["prologue", "switch", "in", "l1", "l2_out", "xchg", "epilogue"]
        phases = {n: round(buf[i] / wgs / (1 if i < 2 else d.denoising_steps)) for i, n in enumerate(names)}
        for i, n in zip(range(11, 16), ["in_mm", "l1_mm", "l2_mm", "out_mm", "publish"]):
            phases[n] = round(buf[i] / wgs / d.denoising_steps)
        phases["wg0_steps"] = [[int(buf[16 + 8 * i + k]) for k in range(1, 7)] for i in range(d.denoising_steps)]
        if hasattr(lib, "dppo_debug_split_xmode"):
            xm = (ctypes.c_uint * 2)()
            lib.dppo_debug_split_xmode(xm, 1)
            m(cond)
            torch.cuda.synchronize()
            lib.dppo_debug_split_xmode(xm, 1)
            phases["groups_shared_l2local"] = [int(xm[0]), int(xm[1])]
    print(json.dumps({"tag": args.tag, "envs": args.envs, "precision": args.precision, "ms_per_launch": ms,
                      "tflops": flops / (ms * 1e-3) / 1e12, "cycles_per_step": phases}), flush=True)


if __name__ == "__main__":
    main()

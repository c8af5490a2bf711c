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
    ap.add_argument("--config-dir", default=os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"))
    ap.add_argument("--config-name", default="ft_ppo_diffusion_mlp_64env")
    ap.add_argument("--tag", default=os.environ.get("DPPO_SAMPLER_QD", "default"))
    args = ap.parse_args()
    import numpy as np
    import torch

    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    dev = torch.device("cuda:0")
    cfg = load_config(args.config_dir, args.config_name, [f"model.precision={args.precision}"])
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
        from diffusionpolicyoptimization_amd import ops
        plan = ops.sampler_plan(d, m.precision, args.envs)
        buf = (ctypes.c_ulonglong * (16 + 64 * 8))()
        lib.dppo_debug_split_cycles(buf, 1)
        n_launch = 20
        e0.record()
        for _ in range(n_launch):
            m(cond)
        e1.record()
        e1.synchronize()
        ms_t = e0.elapsed_time(e1) / n_launch
        lib.dppo_debug_split_cycles(buf, 1)
        G = (args.envs + 15) // 16
        active = G * plan["members"] * plan["sets"]          # workgroups that run steps
        steps = d.denoising_steps // plan["sets"] if plan["kernel"] == 2 else d.denoising_steps   # steps per workgroup
        per = lambda k, n: buf[k] / (n_launch * active * n)
        if plan["kernel"] == 2:   # sample_split4_kernel (folded, P = 2 / 4): XPHASE ids in step order
            names = [(7, "prologue_before_obs_wait", 1), (8, "obs_wait", 1), (0, "prologue_after_obs", 1),
                     (1, "step_head", steps), (11, "in_dense_mfma_u1_store_residual", steps),
                     (2, "in_dense_barrier", steps), (14, "l1_fold_partial_store", steps),
                     (4, "partial_barrier", steps), (15, "publish", steps), (5, "exchange_wait", steps),
                     (6, "epilogue_step_barrier", steps), (9, "loop_end", 1), (10, "done_signal", 1)]
        else:
            names = [(i, f"phase{i}", steps) for i in range(16)]
        phases = {"kernel_plan": plan, "active_workgroups": active, "steps_per_workgroup": steps,
                  "ms_per_launch_timing_build": ms_t, "unit": "shader cycles (s_memtime) of wave 0, per step "
                  "(per launch for the prologue / end phases), averaged over the active workgroups"}
        phases.update({n: round(per(k, cnt), 1) for k, n, cnt in names})
        step_sum = sum(per(k, steps) for k, _, cnt in names if cnt == steps)
        phases["step_total"] = round(step_sum, 1)
        # the shader clock the kernel ran at: the step loop's cycles over its share of the launch time
        phases["wg0_steps_first8phases"] = [[int(buf[16 + 8 * i + k]) for k in range(8)] for i in range(d.denoising_steps)]
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

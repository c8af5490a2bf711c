"""Times the PPO-update kernels in isolation on the bench workload (hopper, bf16, S*E = 32,000
samples, minibatch 50,000 rows): one fused minibatch (loss + gradient) and the old-logprob /
value passes. The row-tile shape comes from DPPO_ROWTILE (see csrc/rowtile.hip).
    python tools/bench_update.py [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=50000)
    args = ap.parse_args()
    import torch

    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    dev = torch.device("cuda:0")
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", [])
    m = instantiate(cfg.model, device=dev, seed=0)
    d = m.dims
    N, kf = 500 * 64, d.ft_denoising_steps
    g = torch.Generator(device=dev).manual_seed(0)
    obs = torch.rand(N, d.sd, device=dev, generator=g) * 2 - 1
    chains = torch.randn(N, kf + 1, d.xd, device=dev, generator=g) * 0.5
    adv = torch.randn(N, device=dev, generator=g)
    ret = torch.randn(N, device=dev, generator=g)
    lp_old = torch.empty(N, kf, device=dev)
    vals = torch.empty(N, device=dev)
    ops.logprob(d, m.precision, m.packed_ft, m.sched, obs, chains, want_elem=False, lp_mean=lp_old)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    mb = timed(lambda: m.minibatch(obs, chains, lp_old, adv, ret, 7, 0, 0, args.rows, global_rows=args.rows), args.reps)
    lp = timed(lambda: ops.logprob(d, m.precision, m.packed_ft, m.sched, obs, chains, want_elem=False, lp_mean=lp_old), 3)
    cv = timed(lambda: ops.critic_forward(d, m.precision, m.packed_critic, obs, values=vals), 5)
    phases = None
    from diffusionpolicyoptimization_amd import _lib
    lib = _lib.load()
    if hasattr(lib, "dppo_debug_phase_cycles"):   # timing build: per-phase cycles of one minibatch
        import ctypes
        buf = (ctypes.c_ulonglong * 32)()
        lib.dppo_debug_phase_cycles(buf, 1)
        m.minibatch(obs, chains, lp_old, adv, ret, 7, 0, 0, args.rows, global_rows=args.rows)
        torch.cuda.synchronize()
        lib.dppo_debug_phase_cycles(buf, 1)
        tiles = (args.rows + 63) // 64
        phases = {f"p{i}": round(buf[i] / tiles) for i in range(11)}
    tb = None
    if hasattr(lib, "dppo_debug_tb_cycles"):   # timing build: the time-MLP backward's phases, one minibatch
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        lib.dppo_debug_tb_cycles(buf, 1)
        m.minibatch(obs, chains, lp_old, adv, ret, 7, 0, 0, args.rows, global_rows=args.rows)
        torch.cuda.synchronize()
        lib.dppo_debug_tb_cycles(buf, 1)
        tb = {f"t{i}": int(buf[i]) for i in range(6)}
    print(json.dumps({"rowtile": "default", "lib": os.path.basename(_lib.LIB_PATH), "time_bwd_cycles": tb,
                      "phase_cycles_per_tile": phases,
                      "minibatch_ms": mb,
                      "logprob_pass_ms": lp, "value_pass_ms": cv,
                      "grad_finite": bool(torch.isfinite(m.grads).all())}), flush=True)


if __name__ == "__main__":
    main()

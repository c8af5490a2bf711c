"""Probe: the actor dW GEMMs of one 50,000-row minibatch (hopper, bf16) through torch.mm
(hipBLASLt) on feature-major images like the row tile writes (XT [K, ldm], DT [N, ldm]):
dW = XT @ DT^T. Prints the per-GEMM and total times (HIP events), for comparison with dw_kernel.
    python tools/probe_dw_blas.py [--rows 50048]"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50048)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M = args.rows
    shapes = {"in": (64, 512), "l1": (512, 512), "l2": (512, 512), "out": (512, 16),
              "c_in": (16, 256), "c_l1": (256, 256), "c_l2": (256, 256), "c_out": (256, 16)}
    g = torch.Generator(device=dev).manual_seed(0)
    ops = {}
    for k, (kx, n) in shapes.items():
        xt = torch.randn(kx, M, device=dev, generator=g).to(torch.bfloat16)
        dt = torch.randn(n, M, device=dev, generator=g).to(torch.bfloat16)
        ops[k] = (xt, dt)
    res = {}
    for dtype_out in ("bf16", "f32"):
        for k, (xt, dt) in ops.items():
            def f():
                if dtype_out == "f32":
                    return torch.mm(xt, dt.t(), out_dtype=torch.float32)
                return torch.mm(xt, dt.t())
            try:
                f()
            except Exception as e:  # out_dtype unsupported
                res[f"{k}_{dtype_out}"] = str(e)[:80]
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                f()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            kx, n = shapes[k]
            res[f"{k}_{dtype_out}"] = {"us": round(ms * 1e3, 2), "tflops": round(2 * kx * n * M / ms / 1e9, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

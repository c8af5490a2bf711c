"""Pretraining step throughput on the reference cfg's shape (hopper, DiffusionMLP 512x3, K = 20,
batch 1024, bf16): one step = c_loss (t, noise draws + dppo_pretrain_minibatch) + AdamW + repack.
    python tools/bench_pretrain.py [--batch 1024] [--steps 50]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    import torch

    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    from diffusionpolicyoptimization_amd.util.optim import AdamW
    cfg = load_config(os.path.join(ROOT, "cfg/gym/pretrain/hopper-medium-v2"), "pre_diffusion_mlp",
                      [f"model.precision={args.precision}"])
    m = instantiate(cfg.model)
    m._pretrain_init()
    opt = AdamW(m.params, 1e-3, weight_decay=1e-6)
    dev = m.device
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.rand(B, 4, 3, device=dev, generator=g) * 2 - 1
    cond = torch.rand(B, 1, 11, device=dev, generator=g) * 2 - 1

    def step():
        loss = m.c_loss(x0, {"state": cond})
        opt.apply_gradients(m.pre_grads)
        m.repack_network()
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        loss = step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    print(json.dumps({"batch": B, "precision": args.precision, "ms_per_step": ms, "samples_per_s": B / ms * 1e3,
                      "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()

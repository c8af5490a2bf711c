"""Times the actor's image re-derivation alone (dppo_pack_all over the fine-tuned actor, the pack
every PPO minibatch's optimizer step ends with) on the bench shape (hopper, bf16): back-to-back
launches bracketed by HIP events on the launch stream.
    python tools/bench_pack.py [--reps 200] [--tag name]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--tag", default="default")
    args = ap.parse_args()
    import torch

    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    dev = torch.device("cuda:0")
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      ["model.precision=bf16"])
    m = instantiate(cfg.model, device=dev, seed=0)
    d, p = m.dims, m.precision
    for _ in range(10):
        ops.pack_all(d, p, m.actor_ft_params, m.packed_ft)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        ops.pack_all(d, p, m.actor_ft_params, m.packed_ft)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"tag": args.tag, "us_per_actor_pack": e0.elapsed_time(e1) * 1e3 / args.reps}))


if __name__ == "__main__":
    main()

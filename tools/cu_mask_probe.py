"""Static CU partitions for the split update, measured without a persistent kernel: the agent's critic
side stream is swapped for a stream created with a CU mask (hipExtStreamCreateWithCUMask), so the
critic's half can occupy only that subset and the actor's latency-bound launches always find the
rest free (VERDICT r05 #1's hypothesis that the two streams' CU contention is what defeated the
fused-tail attempts). Prints the update time per iteration for each mask.
usage: python tools/cu_mask_probe.py [--emulate-ranks 8] [--iters 3] [--masks none,64,96,128]"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from diffusionpolicyoptimization_amd.util.config import get_class, load_config  # noqa: E402


def masked_stream(dev, n_cus, total):
    """A stream on n_cus of the device's CUs, every (total / n_cus)-th one (spread over the XCDs)."""
    hip = ctypes.CDLL("libamdhip64.so")
    step = total // n_cus
    words = [0] * ((total + 31) // 32)
    for c in range(0, total, step):
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--emulate-ranks", type=int, default=1)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--masks", default="none,64,96,128")
    args = ap.parse_args()
    over = ["env.n_envs=64", "train.force_train=True", "train.save_checkpoints=False", "train.save_results=False",
            "train.n_train_itr=1000000", "logdir=/tmp/dppo_cu_mask_probe"]
    if args.emulate_ranks > 1:
        over.append(f"train.emulate_world={args.emulate_ranks}")
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", over)
    agent = get_class(cfg._target_)(cfg)
    dev = agent.device
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    agent.iteration(force_train=True)      # builds the side stream and the bound calls
    plain = agent._side
    for spec in args.masks.split(",") * 2:
        agent._side = plain if spec == "none" else masked_stream(dev, int(spec), total)
        agent.timing.update(rollout_s=0.0, update_s=0.0, n_updates=0, env_steps=0, iters=0)
        torch.cuda.synchronize(dev)
        for _ in range(args.iters):
            agent.iteration(force_train=True)
        torch.cuda.synchronize(dev)
        print(json.dumps({"emulate_ranks": args.emulate_ranks, "critic_cus": spec,
                          "update_ms_per_iter": 1e3 * agent.timing["update_s"] / args.iters,
                          "rollout_ms_per_iter": 1e3 * agent.timing["rollout_s"] / args.iters}), flush=True)
    agent._side = plain


if __name__ == "__main__":
    main()

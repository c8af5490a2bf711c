"""cProfile of one bench iteration's host side (the agent's Python + ctypes calls; the GPU work is
asynchronous, so host time spent waiting shows up in the synchronising calls). For finding host-side
gaps such as the update's start. usage: python tools/host_profile_iteration.py [--top 40]"""
import argparse
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from diffusionpolicyoptimization_amd.util.config import get_class, load_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    over = ["env.n_envs=64", "train.force_train=True", "train.save_checkpoints=False", "train.save_results=False",
            "train.n_train_itr=1000000", "logdir=/tmp/dppo_host_profile"]
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", over)
    agent = get_class(cfg._target_)(cfg)
    agent.iteration(force_train=True)
    pr = cProfile.Profile()
    pr.enable()
    agent.update()
    pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(args.top)
    print(out.getvalue())


if __name__ == "__main__":
    main()

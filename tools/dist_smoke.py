"""Data-parallel agent smoke run (torch.distributed.run, 2+ ranks): a few fine-tuning iterations of
the hopper debug cfg; every rank prints a checksum of its trainable parameters and rank 0 checks
that all replicas stayed identical (the DP step all-reduces gradients, so they must).
    DPPO_DIST_BACKEND=gloo DPPO_SINGLE_DEVICE=1 python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29511 tools/dist_smoke.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    world = int(os.environ.get("WORLD_SIZE", "1"))
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      [f"env.n_envs={4 * world}", "train.n_steps=20", "train.batch_size=200", "train.n_train_itr=3",
                       "train.val_freq=2", "train.save_checkpoints=False", "train.save_results=False",
                       f"logdir=/tmp/dppo_dist_smoke_{os.environ.get('RANK', '0')}"]
                      + os.environ.get("DPPO_SMOKE_OVERRIDES", "").split())
    agent = get_class(cfg._target_)(cfg)
    res = agent.run()
    p = agent.model.train_params.double()
    ck = torch.stack([p.sum(), (p * p).sum()]).cpu()
    parts = [torch.zeros_like(ck) for _ in range(world)]
    dist.all_gather(parts, ck)
    if agent.rank == 0:
        same = all(torch.equal(parts[0], q) for q in parts[1:])
        print(f"dist_smoke world={world} itrs={len(res)} loss={res[1].get('loss')} replicas_identical={same}", flush=True)
        if not same:
            raise SystemExit(f"replicas diverged: {[q.tolist() for q in parts]}")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

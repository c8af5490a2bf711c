"""Data-parallel equivalence worker (torch.distributed.run, 2 ranks; tests/test_agent_gpu.py::
test_data_parallel_update_equals_single_rank_on_the_union). Each rank runs one train iteration
of the reference-batch DP agent (train.dp_scale_batch=false) and, at minibatch 0 of epoch 0, saves
its rollout shard (obs, chains, old log-probs, advantages, returns), its row selection keys and
the all-reduced gradient + metric sums to $DPPO_EQUIV_DIR/rank<r>.npz.
    DPPO_DIST_BACKEND=gloo DPPO_SINGLE_DEVICE=1 DPPO_EQUIV_DIR=/tmp/eq python -m torch.distributed.run \\
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/dp_equiv.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OVERRIDES = ["model.precision=fp32", "env.n_envs=8", "train.n_steps=20", "train.batch_size=400",
             "train.n_train_itr=1", "train.save_checkpoints=False", "train.save_results=False",
             "train.dp_scale_batch=false"]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from diffusionpolicyoptimization_amd.util.config import get_class, load_config
    out_dir = os.environ["DPPO_EQUIV_DIR"]
    rank = int(os.environ.get("RANK", "0"))
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp",
                      OVERRIDES + [f"logdir=/tmp/dppo_equiv_{rank}"])
    a = get_class(cfg._target_)(cfg)

    def hook(epoch, batch, start, rows):
        if (epoch, batch) != (0, 0):
            return
        torch.cuda.synchronize()
        m = a.model
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), obs=a.obs_traj.cpu().numpy(),
                 chains=a.chains_traj.cpu().numpy(), lp_old=a.lp_old.cpu().numpy(), adv=a.adv.cpu().numpy(),
                 ret=a.ret.cpu().numpy(), grads=m.grads.cpu().numpy(), metrics=m.metrics[:5].cpu().numpy(),
                 perm_seed=np.uint64(a.perm_seed), epoch=np.int64(1000 * a.itr), start=np.int64(start),
                 rows=np.int64(rows), n_envs=np.int64(a.n_envs), env_offset=np.int64(a.env_offset),
                 world=np.int64(a.world_size), params=m.train_params.cpu().numpy())
    a.minibatch_hook = hook
    a.iteration(force_train=True)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"rank{rank}_params_end.npy"), a.model.train_params.cpu().numpy())
    dist.barrier()
    if rank == 0:
        print("dp_equiv done", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

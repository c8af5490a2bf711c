"""Child process of test_actor_tail_split_matches_single_launch: one PPO minibatch of 260 64-row
tiles (more than one round of 256 CUs) with the environment's DPPO_ACTOR_TAIL setting; writes the
gradients and metrics to argv[1]."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch

    from diffusionpolicyoptimization_amd import ops
    from tests.helpers import HOPPER, make_models
    from diffusionpolicyoptimization_amd.model.diffusion.sampling import ddpm_buffers
    dev = torch.device("cuda:0")
    d = ops.ModelDims(**HOPPER)
    _, ft, critic = make_models(0, HOPPER)
    pf = torch.tensor(ops.flatten_params(ops.actor_param_spec(d), ft), device=dev)
    pc = torch.tensor(ops.flatten_params(ops.critic_param_spec(d), critic), device=dev)
    tab = torch.tensor(ops.sched_table(ddpm_buffers(d.denoising_steps)), device=dev)
    rng = np.random.default_rng(5)
    N, kf = 2000, d.ft_denoising_steps
    rows = 64 * 260
    T = lambda x: torch.tensor(x, device=dev)
    obs = T(rng.uniform(-1, 1, (N, d.sd)).astype(np.float32))
    chains = T((rng.standard_normal((N, kf + 1, d.xd)) * 0.5).astype(np.float32))
    adv, ret = T(rng.normal(size=N).astype(np.float32)), T(rng.normal(size=N).astype(np.float32))
    packf = ops.pack_actor(d, pf, "bf16")
    _, lpm = ops.logprob(d, "bf16", packf, tab, obs, chains, want_elem=False)
    na, nc = ops.spec_count(ops.actor_param_spec(d)), ops.spec_count(ops.critic_param_spec(d))
    grads = torch.zeros(na + nc, dtype=torch.float32, device=dev)
    metrics = torch.zeros(16, dtype=torch.float64, device=dev)
    ws = ops.ppo_workspace(d, "bf16", rows, dev)
    ops.ppo_minibatch(d, "bf16", ops.ppo_hparams(global_rows=rows), packf, ops.pack_critic(d, pc, "bf16"), pf, tab,
                      obs, chains, lpm, adv, ret, 11, 2, 0, rows, ws, grads, metrics)
    torch.cuda.synchronize()
    np.savez(out, grads=grads.cpu().numpy(), metrics=metrics.cpu().numpy())


if __name__ == "__main__":
    main(sys.argv[1])

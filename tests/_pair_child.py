"""Child of test_pair_sampler_bit_identical: samples 64 envs (bf16, hopper) with the sampler the
environment selects (DPPO_SPLIT_PAIR is read once per process) and saves actions + chains."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, envs):
    import torch

    from diffusionpolicyoptimization_amd import ops
    from diffusionpolicyoptimization_amd.util.config import instantiate, load_config
    dev = torch.device("cuda:0")
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env", [])
    m = instantiate(cfg.model, device=dev, seed=0)
    g = torch.Generator(device=dev).manual_seed(1)
    cond = torch.rand(envs, m.dims.sd, device=dev, generator=g) * 2 - 1
    outs = []
    for det in (False, True):
        s = m(cond, deterministic=det)
        outs += [s.trajectories.cpu().numpy(), s.chains.cpu().numpy()]
    plan = ops.sampler_plan(m.dims, m.precision, envs)
    np.savez(out, *outs, kernel=plan["kernel"])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))

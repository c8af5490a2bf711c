"""Times one optimizer step (dppo_optimizer_step_ex) per variant with HIP events: AdamW + pack
(two launches) against the fused forms (ABI 11), for the actor and the critic ranges."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusionpolicyoptimization_amd import ops  # noqa: E402
from diffusionpolicyoptimization_amd.util.config import instantiate, load_config  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                  ["model.precision=bf16"])
m = instantiate(cfg.model, device="cuda", seed=0)
d = m.dims
for net in ("actor", "actor_l2v", "critic"):
    actor = net != "critic"
    P = m.actor_ft_params if actor else m.critic_params
    img = m.packed_ft if actor else m.packed_critic
    n = P.numel()
    G = torch.randn(n, device="cuda") * 1e-3
    M, V = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    packs = (P, img, None, None) if actor else (None, None, P, img)
    for name, fused, clear in (("adamw+pack", False, False), ("fused", True, False), ("fused+clear", True, True),
                               ("clear-only", False, True)):
        step = ops.BoundOptimizerStep(d, m.precision, P, G, M, V, 0.004, 0.9, 0.999, 1e-7, "keras", *packs,
                                      defer_sampler_tables=actor, l2_from_pl2=net == "actor_l2v",
                                      fused_pack=fused, clear_grads=clear)
        for it in range(5):
            step(it + 1, 1e-6)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for it in range(reps):
            step(it + 6, 1e-6)
        e1.record()
        torch.cuda.synchronize()
        print(f"{net:10s} {name:12s} {e0.elapsed_time(e1) / reps * 1e3:8.1f} us per step", flush=True)

img = m.packed_ft
ops.refresh_sampler_tables(img)
torch.cuda.synchronize()

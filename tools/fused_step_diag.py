"""Which image bytes differ between the fused optimizer step and AdamW + pack (diagnostic)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusionpolicyoptimization_amd import ops  # noqa: E402
from diffusionpolicyoptimization_amd.util.config import instantiate, load_config  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for precision in ("bf16", "fp32"):
    cfg = load_config(os.path.join(ROOT, "cfg/gym/finetune/hopper-v2"), "ft_ppo_diffusion_mlp_64env",
                      [f"model.precision={precision}"])
    m = instantiate(cfg.model, device="cuda", seed=0)
    d = m.dims
    P0, img0 = m.actor_ft_params.clone(), m.packed_ft.clone()
    n = P0.numel()
    gen = torch.Generator(device="cuda").manual_seed(7)
    G0 = torch.randn(n, device="cuda", generator=gen) * 0.05
    M0 = torch.rand(n, device="cuda", generator=gen) * 1e-4
    V0 = torch.rand(n, device="cuda", generator=gen) * 1e-7
    out = {}
    for fused in (False, True):
        P, M, V, img, G = P0.clone(), M0.clone(), V0.clone(), img0.clone(), G0.clone()
        step = ops.BoundOptimizerStep(d, m.precision, P, G, M, V, 0.004, 0.9, 0.999, 1e-7, "keras", P, img, None, None,
                                      defer_sampler_tables=True, fused_pack=fused, clear_grads=fused)
        step(2, 1e-3)
        torch.cuda.synchronize()
        out[fused] = (P.cpu().numpy(), img.cpu().numpy(), G.cpu().numpy())
    a, b = out[False][1], out[True][1]
    print(precision, "params equal", np.array_equal(out[False][0], out[True][0]), "grads zero", not out[True][2].any())
    dif = np.nonzero(a != b)[0]
    print(precision, "differing bytes", dif.size, "of", a.size)
    if dif.size:
        runs = np.split(dif, np.nonzero(np.diff(dif) > 1)[0] + 1)
        for r in runs[:12]:
            print("  run", int(r[0]), int(r[-1]), "len", r.size)
        print("  runs", len(runs))
        nz0 = np.nonzero(a != img0.cpu().numpy())[0]
        nz1 = np.nonzero(b != img0.cpu().numpy())[0]
        print("  changed vs initial: unfused", nz0.size, "fused", nz1.size)

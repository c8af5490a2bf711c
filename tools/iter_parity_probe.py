"""Whole-iteration parity numbers of one seed without the test's asserts (tests/test_iteration_gpu.py's
comparison, every quantity printed): for telling fp noise in the loss metrics from a kernel error.
usage: python tools/iter_parity_probe.py <seed> [--repeat N]    (DPPO_LIB selects the library)"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_iteration_gpu as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seed", type=int)
    ap.add_argument("--repeat", type=int, default=1)
    args = ap.parse_args()
    for rep in range(args.repeat):
        with tempfile.TemporaryDirectory() as tmp:
            a, orc = T._agent_and_oracle(args.seed, tmp)
            for it in range(3):
                p0 = a.model.train_params.cpu().numpy().astype(np.float64)
                th0 = orc.theta.copy()
                res, ref = a.iteration(), orc.iteration()
                ch = a.chains_traj.cpu().numpy().reshape(ref["chains"].shape)
                e = {"rep": rep, "itr": it, "eval": bool(res["eval"]),
                     "chains_abs": float(np.abs(ch - ref["chains"]).max())}
                if not res["eval"]:
                    last = ref["metrics"][-1]
                    for k in ("pg_loss", "v_loss", "approx_kl", "clipfrac"):
                        e[k] = (float(res[k]), float(last.get(k, float("nan"))))
                    dg = a.model.train_params.cpu().numpy().astype(np.float64) - p0
                    dr = orc.theta - th0
                    diff = np.abs(dg - dr)
                    scale = np.abs(dr).max()
                    e["param_delta_l2_rel"] = float(np.linalg.norm(dg - dr) / np.linalg.norm(dr))
                    e["param_delta_p99_rel"] = float(np.quantile(diff, 0.99) / scale)
                    e["lp_old_abs"] = float(np.abs(a.lp_old.cpu().numpy() - ref["lp_old"]).max())
                print(json.dumps(e), flush=True)


if __name__ == "__main__":
    main()

"""How well-conditioned is the whole-iteration comparison? The float64 oracle of
tests/test_iteration_gpu.py run twice from the same state, one copy's parameters perturbed at fp32
rounding level (relative 2^-24 per element) before a training iteration: the spread of its loss
metrics and parameter update is what any fp32 implementation can be held to on that seed.
usage: python tools/oracle_sensitivity.py <seed> [--perturb-at 2] [--trials 3]   (needs a GPU for the
agent that seeds the oracle's weights; the oracle itself is NumPy)"""
import argparse
import copy
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
    ap.add_argument("--perturb-at", type=int, default=2)
    ap.add_argument("--trials", type=int, default=3)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        _, orc = T._agent_and_oracle(args.seed, tmp)
        for _ in range(args.perturb_at):
            orc.iteration()
        base = copy.deepcopy(orc)
        th0 = base.theta.copy()
        ref = base.iteration()
        dref = base.theta - th0
        last = ref["metrics"][-1]
        print(json.dumps({"seed": args.seed, "itr": args.perturb_at, "pg_loss": last["pg_loss"],
                          "v_loss": last["v_loss"], "n_minibatches": len(ref["metrics"])}), flush=True)
        rng = np.random.default_rng(0)
        for trial in range(args.trials):
            o = copy.deepcopy(orc)
            o.theta = o.theta * (1.0 + 2.0 ** -24 * rng.standard_normal(o.theta.shape))
            t0 = o.theta.copy()
            r = o.iteration()
            d = o.theta - t0
            lt = r["metrics"][-1]
            print(json.dumps({
                "trial": trial,
                "pg_loss_rel": abs(lt["pg_loss"] - last["pg_loss"]) / abs(last["pg_loss"]),
                "v_loss_rel": abs(lt["v_loss"] - last["v_loss"]) / abs(last["v_loss"]),
                "param_delta_l2_rel": float(np.linalg.norm(d - dref) / np.linalg.norm(dref)),
                "param_delta_p99_rel": float(np.quantile(np.abs(d - dref), 0.99) / np.abs(dref).max()),
                "n_minibatches": len(r["metrics"])}), flush=True)


if __name__ == "__main__":
    main()

#!/bin/bash
# A/B of the split sampler's members per group (DPPO_SPLIT_P=4 default vs 8), bench workload
# (hopper, bf16, 64 envs): HIP-event time per launch, interleaved twice. Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
for p in 4 8 4 8; do
  echo -n "P=$p "
  DPPO_SPLIT_P=$p timeout -k 5 120 python tools/bench_sampler.py --tag p$p --reps 300 | cut -c1-160 || exit 1
done
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/sampler_p4.npy"); b = np.load("gpurun_out/sampler_p8.npy")
print("P4 vs P8 actions: max|diff| %.3g  max|a| %.3g" % (np.abs(a - b).max(), np.abs(b).max()))
PY

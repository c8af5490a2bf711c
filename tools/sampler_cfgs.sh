#!/bin/bash
# Times every sampler geometry (DPPO_SAMPLER_CFG) and checks they produce identical actions.
#   tools/sampler_cfgs.sh [cfgs...]   (default: s e i q r)
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cfgs=${@:-s e i q r}
for c in $cfgs; do
    DPPO_SAMPLER_CFG=$c timeout -k 10 300 python tools/bench_sampler.py --tag cfg_$c
done
python - $cfgs <<'PY'
import sys, numpy as np
c = sys.argv[1:]
ref = np.load(f"gpurun_out/sampler_cfg_{c[0]}.npy")
for x in c[1:]:
    y = np.load(f"gpurun_out/sampler_cfg_{x}.npy")
    print(x, "max|diff| vs", c[0], float(np.abs(y - ref).max()))
PY

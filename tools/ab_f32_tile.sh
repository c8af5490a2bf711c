#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2 3; do for v in main f32w16; do
  if [ $v = main ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
  log=gpurun_out/abf32_${v}_$r.log
  DPPO_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --precision fp32 > $log 2>&1 || { echo "bench $v failed"; tail -20 $log; exit 1; }
  python - $log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), "ms/it", round(d["ms_per_step"], 2), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4),
      "roll_ms", round(1e3 * d["rollout_s_per_iter"], 2), "upd_ms", round(1e3 * d["update_s_per_iter"], 2))
PY
done; done

#!/bin/bash
# Agent-bench A/B of the main library against lib/variants/libdppo_hip_<tag>.so, alternating, at N = 1
# and on the emulated W = 8 rank, each run time-limited. usage: tools/ab_bench_lib.sh <tag> [pairs]
set -o pipefail
tag=$1; pairs=${2:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 $pairs); do
  for v in main $tag; do
    if [ $v = main ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    for emu in 1 8; do
      log=gpurun_out/abl_${tag}_${v}_emu${emu}_$r.log
      DPPO_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks $emu > $log 2>&1 \
        || { echo "bench $v emu$emu failed"; tail -20 $log; exit 1; }
      python - $log $v $emu <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "emu" + sys.argv[3], round(d["value"]), "ms/it", round(d["ms_per_step"], 2), "mb_ms",
      round(d["ppo_minibatch_avg_ms"], 4), "roll_ms", round(1e3 * d["rollout_s_per_iter"], 2), "upd_ms",
      round(1e3 * d["update_s_per_iter"], 2))
PY
    done
  done
done

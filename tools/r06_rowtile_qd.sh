#!/bin/bash
# the row tiles' weight-queue depth (DPPO_ROWTILE_QD, default 3) at 2 and 4: agent bench at N = 1 and on
# the emulated W = 8 rank, alternating libraries, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2; do
  for v in main qd2 qd4; do
    if [ $v = main ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    for emu in 1 8; do
      log=gpurun_out/qd_${v}_emu${emu}_$r.log
      DPPO_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --emulate-ranks $emu > $log 2>&1 \
        || { echo "bench $v emu$emu failed"; tail -20 $log; exit 1; }
      python - $log $v $emu <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "emu" + sys.argv[3], round(d["value"]), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4), "upd_ms",
      round(1e3 * d["update_s_per_iter"], 2))
PY
    done
  done
done

#!/bin/bash
# same-box A/B of the env pool's solo floor on the wrapper-stack env (trivial simulator, 1 and 4 host
# threads): DPPO_ENV_SOLO_FLOOR_US = 0 (always the pool) vs the default 25 us. usage: tools/ab_lowdim_solo.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for thr in 1 4; do
    for fl in 0 25; do
      log=gpurun_out/ab_solo_t${thr}_f${fl}_$r.log
      DPPO_ENV_SOLO_FLOOR_US=$fl timeout -k 10 300 python -u bench.py --env lowdim --env-threads $thr --no-cpu-baseline --steps 3 --warmup 1 > $log 2>&1 || { tail -20 $log; exit 1; }
      python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('threads $thr floor $fl', round(d['value']), 'roll_ms', round(d['rollout_s_per_iter']*1e3,2), 'upd_ms', round(d['update_s_per_iter']*1e3,2))"
    done
  done
done

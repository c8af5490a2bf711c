#!/bin/bash
# same-box A/B: deferred split-sampler tables (DPPO_DEFER_TABLES=1, default) vs packing them at every
# optimizer step (=0), alternating runs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 0; do
    DPPO_DEFER_TABLES=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abdefer_${v}_$i.log 2>&1 || { tail -20 gpurun_out/abdefer_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abdefer_${v}_$i.log').read().strip().splitlines()[-1]); print('defer=$v', round(d['value']), round(d['update_s_per_iter']*1e3,2), round(d['ppo_minibatch_avg_ms'],4), round(d['rollout_s_per_iter']*1e3,2))"
  done
done

#!/bin/bash
# same-box A/B of an environment knob on the bench: tools/ab_env.sh VAR "A B" [rounds] [extra bench args]
# (e.g. --emulate-ranks 8)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
var=$1; vals=$2; n=${3:-2}; shift 3 2>/dev/null; extra="$*"; sfx=$(echo "$extra" | tr -cd 'a-z0-9')
for i in $(seq 1 $n); do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $extra > gpurun_out/ab_${var}_${v}${sfx}_$i.log 2>&1 || { tail -20 gpurun_out/ab_${var}_${v}${sfx}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${var}_${v}${sfx}_$i.log').read().strip().splitlines()[-1]); print('$var=$v $extra', round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4), 'roll', round(d['rollout_s_per_iter']*1e3,2))"
  done
done

#!/bin/bash
# A/B of an environment knob on bench.py (no CPU baseline), alternating A B A B.
# usage: tools/ab_env.sh VAR valA valB [bench args]
set -o pipefail
var=$1; a=$2; b=$3; shift 3
for v in $a $b $a $b; do
  env $var=$v timeout -k 5 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_env_$v.json || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_env_$v.json')); print('$var=$v', round(d['value']), 'roll', round(1e3*d['rollout_s_per_iter'],2), 'upd', round(1e3*d['update_s_per_iter'],2), 'mb', round(d['ppo_minibatch_avg_ms'],4))"
done

#!/bin/bash
# Update-phase knobs on top of DPPO_ACTOR_TAIL=0 (bench.py, hopper 64 envs).
set -o pipefail
mkdir -p gpurun_out
run() { echo -n "$1: "; env DPPO_ACTOR_TAIL=0 $2 timeout -k 5 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abk.log 2>&1 || { tail -5 gpurun_out/abk.log; exit 1; }; tail -1 gpurun_out/abk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f update %.2f ms rollout %.2f ms mb %.3f ms' % (d['value'], d['update_s_per_iter']*1e3, d['rollout_s_per_iter']*1e3, d['ppo_minibatch_avg_ms']))"; }
run notail "X=1"
run a64x8 "DPPO_ROWTILE=64x8"
run c32x8 "DPPO_ROWTILE=64x16,32x8"
run zero64 "DPPO_ZERO_BLOCKS=64"
run tk128 "DPPO_DW_TK=128"
run notail "X=1"

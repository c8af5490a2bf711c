#!/bin/bash
# Update-phase time per iteration (bench.py, hopper 64 envs) under the update scheduling knobs.
set -o pipefail
mkdir -p gpurun_out
run() { echo -n "$1: "; env $2 timeout -k 5 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abk.log 2>&1 || { tail -5 gpurun_out/abk.log; exit 1; }; tail -1 gpurun_out/abk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f update %.2f ms rollout %.2f ms mb %.3f ms' % (d['value'], d['update_s_per_iter']*1e3, d['rollout_s_per_iter']*1e3, d['ppo_minibatch_avg_ms']))"; }
run default "X=1"
run nosplit "DPPO_SPLIT_UPDATE=0"
run notail "DPPO_ACTOR_TAIL=0"
run default "X=1"

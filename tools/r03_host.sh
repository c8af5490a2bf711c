#!/bin/bash
# r03: GPU tests, the bench line and the emulated W = 8 rank line (host enqueue time per minibatch)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
for mode in "" "--emulate-ranks 8"; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $mode > gpurun_out/host_$tag.log 2>&1 || { tail -20 gpurun_out/host_$tag.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/host_$tag.log').read().strip().splitlines()[-1])
print('$mode', round(d['value']), 'roll', round(d['rollout_s_per_iter']*1e3,2), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4), {k: round(v,1) for k,v in d['host_us_per_minibatch'].items()})"
done

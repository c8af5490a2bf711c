#!/bin/bash
# r03: launch-event ring in the rollout: GPU tests, two bench runs, the HIP trace of the rollout -> update gap
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_evring.log 2>&1 || { tail -40 gpurun_out/gpu_tests_evring.log; exit 1; }
tail -1 gpurun_out/gpu_tests_evring.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_evring_$i.log 2>&1 || { tail -20 gpurun_out/bench_evring_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_evring_$i.log').read().strip().splitlines()[-1]); print(round(d['value']), 'ms', round(d['ms_per_step'],2), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4), 'roll', round(d['rollout_s_per_iter']*1e3,2))"
done
bash tools/r03_hiptrace.sh

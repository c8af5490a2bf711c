#!/bin/bash
# r03: bucket-parallel time_bwd: GPU tests, same-box bench A/B at N=1 and for the emulated W=8 rank
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_tbm.log 2>&1 || { tail -40 gpurun_out/gpu_tests_tbm.log; exit 1; }
tail -1 gpurun_out/gpu_tests_tbm.log
DPPO_TIME_BWD_MULTI=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "minibatch_grads or full_size or l2_deferred" > gpurun_out/gpu_tests_tbm1.log 2>&1 || { tail -30 gpurun_out/gpu_tests_tbm1.log; exit 1; }
tail -1 gpurun_out/gpu_tests_tbm1.log
bash tools/ab_env.sh DPPO_TIME_BWD_MULTI "1 0" 2
for v in 1 0; do
  DPPO_TIME_BWD_MULTI=$v timeout -k 10 300 python -u bench.py --emulate-ranks 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/emu_tbm_$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/emu_tbm_$v.log').read().strip().splitlines()[-1]); print('emu8 tbm=$v', round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4))"
done

#!/bin/bash
# r03: GPU tests, then same-box A/B of the deferred l2 gradient (DPPO_L2_DEFER 1 vs 0): bench + emulated W=8 rank
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
bash tools/ab_env.sh DPPO_L2_DEFER "1 0" 2 || exit 1
for v in 1 0 1 0; do
  DPPO_L2_DEFER=$v timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --emulate-ranks 8 > gpurun_out/l2d_emu_$v.log 2>&1 || { tail -20 gpurun_out/l2d_emu_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/l2d_emu_$v.log').read().strip().splitlines()[-1])
print('emu8 l2defer=$v', round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4))"
done

#!/bin/bash
# r03: GPU tests, then a bench line and an iteration kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03k}
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
timeout -k 10 800 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$tag.log').read().strip().splitlines()[-1]); print(round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4), 'roll', round(d['rollout_s_per_iter']*1e3,2), 'samp', d['roofline']['avg_launch_ms'])"
bash tools/profile.sh $tag --steps 2 --warmup 1 || exit 1
echo done

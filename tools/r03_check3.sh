#!/bin/bash
# r03: GPU tests, a bench line, an iteration kernel trace (profiles/r03_iteration_kernel_stats.csv source)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03e}
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
timeout -k 10 800 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
DPPO_EARLY_DW=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_noearly_$tag.log 2>&1 || { tail -30 gpurun_out/bench_noearly_$tag.log; exit 1; }
tail -1 gpurun_out/bench_noearly_$tag.log
bash tools/profile.sh $tag --steps 2 --warmup 1 || exit 1
echo done

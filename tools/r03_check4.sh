#!/bin/bash
# r03: GPU tests, a bench line, the isolated update kernels (bench_update under a kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03g}
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
timeout -k 10 800 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bu_$tag -o run -- python3 -u $GRAFT_REPO_ROOT/tools/bench_update.py --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/bu_$tag.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/bu_$tag.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bu_$tag.log
echo done

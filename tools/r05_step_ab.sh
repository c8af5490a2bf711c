#!/bin/bash
# The one-launch actor step: its tests, its time alone (tools/bench_step.py) and the agent A/B against
# the r04 step (DPPO_FUSED_STEP = all / critic) at N = 1 and on the emulated W = 8 rank, each step
# time-limited. usage: tools/r05_step_ab.sh <tag>   TESTS=<pytest -k expr>, PAIRS=<n> (default 1)
set -o pipefail
tag=${1:-step}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTS" \
    > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_$tag.log
fi
timeout -k 10 300 python -u tools/bench_step.py > gpurun_out/bench_step_$tag.txt 2>&1 || { echo "bench_step failed"; tail -20 gpurun_out/bench_step_$tag.txt; exit 1; }
grep "us per step" gpurun_out/bench_step_$tag.txt
NOTESTS=1 PAIRS=${PAIRS:-1} bash tools/r05_check.sh $tag

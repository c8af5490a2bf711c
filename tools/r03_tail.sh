#!/bin/bash
# r03: GPU tests, then same-box A/B of the short-last-round overlap (DPPO_TAIL_OVERLAP) on the bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=${1:-tail}
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
for v in 1 0; do DPPO_TAIL_OVERLAP=$v timeout -k 10 200 python tools/bench_update.py --reps 20 > gpurun_out/bu_${tag}_$v.log 2>&1 || exit 1; echo "overlap=$v"; tail -1 gpurun_out/bu_${tag}_$v.log | cut -c1-300; done
bash tools/ab_env.sh DPPO_TAIL_OVERLAP "1 0" 2

#!/bin/bash
# r03: the lowdim-env agent test, a bench line, an iteration kernel trace and the update kernels' PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_iteration_gpu.py -k lowdim -m gpu > gpurun_out/r03b_tests.log 2>&1 || { tail -40 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03b.log 2>&1 || { tail -30 gpurun_out/bench_r03b.log; exit 1; }
tail -1 gpurun_out/bench_r03b.log
bash tools/profile.sh r03b --steps 2 --warmup 1 || exit 1
bash tools/pmc_sq_update.sh r03b || exit 1
bash tools/pmc_update.sh r03b || exit 1
echo done

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log

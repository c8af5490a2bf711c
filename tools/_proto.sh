set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_agent_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/agent_tests.log 2>&1; rc=$?
tail -8 gpurun_out/agent_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/agent_tests.log; exit $rc; }
for p in tagged go; do
  DPPO_ROLLOUT_PROTOCOL=$p timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$p.log 2>&1 || { tail -20 gpurun_out/bench_$p.log; exit 1; }
  echo $p; tail -1 gpurun_out/bench_$p.log
done

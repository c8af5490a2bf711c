set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_agent_gpu.py tests/test_host_cpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/actab_tests.log 2>&1; rc=$?
tail -2 gpurun_out/actab_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/actab_tests.log; exit $rc; }
for r in 1 2; do
  (cd _abbase && timeout -k 10 200 python -u bench.py --no-cpu-baseline > ../gpurun_out/actab_base$r.log 2>&1) || { tail -20 gpurun_out/actab_base$r.log; exit 1; }
  echo base$r; tail -1 gpurun_out/actab_base$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('rollout_s_per_iter'), d.get('update_s_per_iter'))"
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/actab_new$r.log 2>&1 || { tail -20 gpurun_out/actab_new$r.log; exit 1; }
  echo new$r; tail -1 gpurun_out/actab_new$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('rollout_s_per_iter'), d.get('update_s_per_iter'))"
done

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grad or agent" > gpurun_out/t.log 2>&1; rc=$?
tail -2 gpurun_out/t.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/t.log; exit $rc; }
for r in 1 2; do
for v in 16 256 4; do
DPPO_ZERO_BLOCKS=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
echo zb=$v $(tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['rollout_s_per_iter'], d['update_s_per_iter'])")
done
done

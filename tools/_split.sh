set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/all.log 2>&1; rc=$?
tail -3 gpurun_out/all.log
[ $rc -eq 0 ] || { tail -50 gpurun_out/all.log; exit $rc; }
for f in 1 0 1 0; do
DPPO_SPLIT_UPDATE=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
echo split=$f $(tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['rollout_s_per_iter'], d['update_s_per_iter'], d['ppo_minibatch_avg_ms'])")
done

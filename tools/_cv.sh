set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for v in "64x16,32x8o4" "64x16,32x8"; do
DPPO_ROWTILE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
echo rt=$v $(tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['rollout_s_per_iter'], d['update_s_per_iter'])")
done
done

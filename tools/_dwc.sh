set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for v in 0 3 6; do
if [ $v = 0 ]; then unset DPPO_DW_CHUNKS; else export DPPO_DW_CHUNKS=$v; fi
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
echo dwc=$v $(tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['rollout_s_per_iter'], d['update_s_per_iter'])")
done
done

set -o pipefail
cd /tmp && export TMPDIR=/tmp
for v in default tb256 tb512; do
if [ $v = default ]; then unset DPPO_LIB; else export DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
rm -rf $GRAFT_REPO_ROOT/gpurun_out/tb_$v
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tb_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/tb_$v.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/tb_$v/run_kernel_stats.csv')):
    if 'time_bwd' in r['Name']: print('$v', r['Calls'], round(float(r['AverageNs'])/1000,2))
"
done

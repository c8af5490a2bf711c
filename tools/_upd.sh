set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grad or minibatch or update or agent or time" > gpurun_out/upd_tests.log 2>&1; rc=$?
tail -2 gpurun_out/upd_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/upd_tests.log; exit $rc; }
timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu.log 2>&1 || { tail -20 gpurun_out/bu.log; exit 1; }
tail -1 gpurun_out/bu.log
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/uprof_$1; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/uprof_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/uprof_$1 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/uprof_$1/log 2>&1 || exit $?
python3 -c "
import csv
for r in list(csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/uprof_$1/run_kernel_stats.csv')))[:9]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))
"

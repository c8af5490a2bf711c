set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DPPO_ROWTILE=64x8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grad or minibatch" > gpurun_out/rt_tests.log 2>&1; rc=$?
tail -2 gpurun_out/rt_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/rt_tests.log; exit $rc; }
for r in 1 2; do
for t in 64x16 64x8; do
DPPO_ROWTILE=$t timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu_$t.log 2>&1 || { tail -20 gpurun_out/bu_$t.log; exit 1; }
echo $t; tail -1 gpurun_out/bu_$t.log | cut -c1-200
done
done
for t in 64x16 64x8; do
DPPO_ROWTILE=$t DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_rtime.so timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bur_$t.log 2>&1 || { tail -20 gpurun_out/bur_$t.log; exit 1; }
echo $t; tail -1 gpurun_out/bur_$t.log | cut -c1-300
done

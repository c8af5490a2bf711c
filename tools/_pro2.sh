set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "grad or minibatch or agent or tail or pretrain or logprob" > gpurun_out/t.log 2>&1; rc=$?
tail -2 gpurun_out/t.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/t.log; exit $rc; }
for r in 1 2; do
for v in default base; do
if [ $v = base ]; then export DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_base.so; else unset DPPO_LIB; fi
timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu.log 2>&1 || { tail -20 gpurun_out/bu.log; exit 1; }
echo $v $(tail -1 gpurun_out/bu.log | cut -c40-110)
done
done

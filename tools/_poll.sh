set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sampl or pipelined or smoke or rollout" > gpurun_out/samp_tests.log 2>&1; rc=$?
tail -2 gpurun_out/samp_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/samp_tests.log; exit $rc; }
for r in 1 2; do
timeout -k 10 120 python -u tools/bench_sampler.py > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
tail -1 gpurun_out/bs.log | cut -c1-120
DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_poll1.so timeout -k 10 120 python -u tools/bench_sampler.py --tag poll1 > gpurun_out/bs1.log 2>&1 || { tail -20 gpurun_out/bs1.log; exit 1; }
tail -1 gpurun_out/bs1.log | cut -c1-120
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s.log 2>&1 || { tail -20 gpurun_out/bench_s.log; exit 1; }
tail -1 gpurun_out/bench_s.log | cut -c1-300

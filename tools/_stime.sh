set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_stime.so timeout -k 10 120 python -u tools/bench_sampler.py --tag stime > gpurun_out/stime.log 2>&1 || { tail -20 gpurun_out/stime.log; exit 1; }
tail -1 gpurun_out/stime.log | cut -c1-900

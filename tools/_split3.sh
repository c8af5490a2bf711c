set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "sampler" -x -q --timeout 120 --timeout-method thread > gpurun_out/split_t.log 2>&1; rc=$?
tail -2 gpurun_out/split_t.log
[ $rc -eq 0 ] || exit $rc
for E in 64 512; do timeout -k 10 120 python tools/bench_sampler.py --envs $E --tag x$E || exit 1; done
DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_stime.so timeout -k 10 120 python tools/bench_sampler.py --envs 64 --tag t64

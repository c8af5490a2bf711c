set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/round_check.sh r03t || exit 1
bash tools/variant_build.sh tim "-DDPPO_SAMPLER_TIMING" > gpurun_out/vb_tim.log 2>&1 || exit 1
DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_tim.so timeout -k 5 120 python tools/bench_sampler.py --tag tim > gpurun_out/tim_r03t.json || exit 1
cat gpurun_out/tim_r03t.json | cut -c1-1500

set -e
timeout -k 10 600 tools/sampler_cfgs.sh s r > gpurun_out/cfgs.log 2>&1
for c in s r; do DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_stime.so DPPO_SAMPLER_CFG=$c timeout -k 10 120 python tools/bench_sampler.py --tag t_$c >> gpurun_out/cfgs.log 2>&1; done
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_agent_gpu.py -k "sampl or pipelined or bound" -x -q > gpurun_out/t.log 2>&1
DPPO_SAMPLER_CFG=r timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_agent_gpu.py -k "sampl or pipelined or bound" -x -q >> gpurun_out/t.log 2>&1

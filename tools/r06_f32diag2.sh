#!/bin/bash
# seed-44 iteration parity numbers: the 8-member fp32 sampler twice, the 4-member build once
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/iter_parity_probe.py 44 --repeat 2 > gpurun_out/probe44_p8.log 2>&1 || { tail -20 gpurun_out/probe44_p8.log; exit 1; }
grep '^{' gpurun_out/probe44_p8.log
DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_f32p4.so timeout -k 10 300 python -u tools/iter_parity_probe.py 44 > gpurun_out/probe44_p4.log 2>&1 || { tail -20 gpurun_out/probe44_p4.log; exit 1; }
grep '^{' gpurun_out/probe44_p4.log

#!/bin/bash
# r03: actor row-tile phase cycles (timing build) + isolated update kernels
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
DPPO_LIB=$V/libdppo_hip_rtim.so timeout -k 10 180 python -u tools/bench_update.py --reps 5 > gpurun_out/tim_rtim2.log 2>&1 || { tail -20 gpurun_out/tim_rtim2.log; exit 1; }
tail -1 gpurun_out/tim_rtim2.log
timeout -k 10 180 python -u tools/bench_update.py --reps 10 > gpurun_out/bu_plain.log 2>&1 || { tail -20 gpurun_out/bu_plain.log; exit 1; }
tail -1 gpurun_out/bu_plain.log

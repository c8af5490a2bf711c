#!/bin/bash
# r03: phase-cycle timing builds (tools/variant_build.sh): the split sampler (stim) and the
# update row tiles (rtim), plus the plain update / sampler timings for reference
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
DPPO_LIB=$V/libdppo_hip_stim.so timeout -k 10 180 python -u tools/bench_sampler.py --tag stim > gpurun_out/tim_stim.log 2>&1 || { tail -20 gpurun_out/tim_stim.log; exit 1; }
tail -1 gpurun_out/tim_stim.log
DPPO_LIB=$V/libdppo_hip_rtim.so timeout -k 10 180 python -u tools/bench_update.py --reps 5 > gpurun_out/tim_rtim.log 2>&1 || { tail -20 gpurun_out/tim_rtim.log; exit 1; }
tail -1 gpurun_out/tim_rtim.log
echo done

#!/bin/bash
# r03: pipelined-rollout phase split (timing build) + the emulated W = 8 rank bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
DPPO_LIB=$V/libdppo_hip_stim.so timeout -k 10 240 python -u tools/rollout_probe.py > gpurun_out/rprobe.log 2>&1 || { tail -20 gpurun_out/rprobe.log; exit 1; }
tail -1 gpurun_out/rprobe.log
timeout -k 10 400 python -u bench.py --emulate-ranks 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_emu8.log 2>&1 || { tail -20 gpurun_out/bench_emu8.log; exit 1; }
tail -1 gpurun_out/bench_emu8.log
echo done

#!/bin/bash
# r03: GPU tests, a bench line, then the sampler and row-tile phase timers (timing variants)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03d}
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
timeout -k 10 800 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_stim.so timeout -k 10 120 python -u tools/bench_sampler.py --tag stim_$tag --reps 50 > gpurun_out/samp_stim_$tag.log 2>&1 || { tail -20 gpurun_out/samp_stim_$tag.log; exit 1; }
tail -1 gpurun_out/samp_stim_$tag.log
DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_rtim.so timeout -k 10 200 python -u tools/bench_update.py --reps 5 > gpurun_out/upd_rtim_$tag.log 2>&1 || { tail -20 gpurun_out/upd_rtim_$tag.log; exit 1; }
tail -1 gpurun_out/upd_rtim_$tag.log

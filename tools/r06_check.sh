#!/bin/bash
# Round-6 check: GPU tests (TESTS=<-k expr> narrows them), the default bench line and the emulated
# W = 8 rank's line; PHASES=1 adds the folded sampler's phase profile (timing build lib/variants/
# libdppo_hip_stim.so), TRACE=1 the emulated rank's kernel trace + timeline.
# usage: tools/r06_check.sh <tag>
set -o pipefail
tag=${1:-r06}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log | cut -c1-600
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/${tag}_emu8.log 2>&1 || { tail -20 gpurun_out/${tag}_emu8.log; exit 1; }
tail -1 gpurun_out/${tag}_emu8.log | cut -c1-600
if [ -n "$PHASES" ]; then
  DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_stim.so timeout -k 10 200 \
    python -u tools/bench_sampler.py --reps 100 --tag stim > gpurun_out/${tag}_sampler_phases.json 2>&1 || { tail -20 gpurun_out/${tag}_sampler_phases.json; exit 1; }
  tail -1 gpurun_out/${tag}_sampler_phases.json | cut -c1-900
fi
if [ -n "$TRACE" ]; then
  timeout -k 10 700 bash tools/emu_trace.sh $tag || exit 1
  head -60 gpurun_out/prof_emu_$tag/timeline.txt
fi

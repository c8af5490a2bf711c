#!/bin/bash
# Round-6 first check: the new parity cases (XD = 8 gradients, config 2 at full size, walker2d on the
# folded sampler), then the default bench line, walker2d 256 envs, and the emulated W = 8 rank's line.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "narrow or full_size or ppo_minibatch_grads or sampler_bf16_sizes or sampler_injected or logprob" > gpurun_out/r06a_tests.log 2>&1 || { tail -40 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06a_bench.log 2>&1 || { tail -20 gpurun_out/r06a_bench.log; exit 1; }
tail -1 gpurun_out/r06a_bench.log | cut -c1-400
ONLY=walker256 NOPROF=1 timeout -k 10 400 bash tools/r05_configs.sh r06a || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/r06a_emu8.log 2>&1 || { tail -20 gpurun_out/r06a_emu8.log; exit 1; }
tail -1 gpurun_out/r06a_emu8.log | cut -c1-400

#!/bin/bash
# the episode accounting kernel with batched loads: its parity tests and the agent tests that read it,
# then the default bench line and the kernel's time in a short trace
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "episode or test_agent_iterations or test_iterations_match_oracle" > gpurun_out/ep_tests.log 2>&1 || { tail -30 gpurun_out/ep_tests.log; exit 1; }
tail -1 gpurun_out/ep_tests.log
bash tools/profile.sh r06ep --steps 2 --warmup 1 || { tail -20 gpurun_out/prof_r06ep/bench.log; exit 1; }
grep -h "episode_sums" gpurun_out/prof_r06ep/run_kernel_stats.csv | cut -d, -f1-6

#!/bin/bash
# HIP API + memory-copy + kernel trace of a short bench run (no counters): what the host does
# between the rollout's last sampler launch and the update's first kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/hipt_r03
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/bench.log 2>&1

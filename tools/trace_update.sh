#!/bin/bash
# Kernel trace of tools/bench_update.py (fused minibatch) and of a short agent update (split
# minibatches on two streams), then the timeline of the last dispatches of each.
# usage: tools/trace_update.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/utrace_$tag
mkdir -p $base/mb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $base/mb -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 10 > $base/mb/log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py $base/mb/run_kernel_trace.csv 30 > $base/mb_timeline.txt

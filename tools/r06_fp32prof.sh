#!/bin/bash
# kernel trace + stats of one fp32 bench iteration (hopper 64 envs, the reference's precision)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/fp32prof
mkdir -p $base
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $base -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32 --steps 1 --warmup 1 --no-cpu-baseline > $base/log 2>&1 || { tail -20 $base/log; exit 1; }
tail -1 $base/log | cut -c1-200

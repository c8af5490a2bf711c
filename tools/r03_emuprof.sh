#!/bin/bash
# r03: kernel trace of the emulated W = 8 rank (one rank's share of the 8-GPU update)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/prof_emu_$1
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --emulate-ranks 8 --steps 2 --warmup 1 > $out/bench.log 2>&1

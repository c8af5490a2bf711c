#!/bin/bash
# kernel trace of the emulated W = 8 rank (one rank's share of the 8-GPU update), then its timeline
# usage: tools/emu_trace.sh <tag> [extra env assignments for bench.py, e.g. DPPO_X=1]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/prof_emu_$tag
mkdir -p $out
env "$@" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --emulate-ranks 8 --steps 2 --warmup 1 > $out/bench.log 2>&1 || exit $?
f=$(ls $out/*kernel_trace.csv $out/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $GRAFT_REPO_ROOT/tools/mb_timeline.py $f 40 > $out/timeline.txt
tail -1 $out/bench.log | cut -c1-400

#!/bin/bash
# PMC passes over tools/bench_update.py (one counter group per pass, kernel-trace only).
# usage: tools/pmc_update.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "$@"; do
    out=$GRAFT_REPO_ROOT/gpurun_out/pmcu_${tag}_$i
    mkdir -p $out
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $out/log 2>&1 || exit $?
    i=$((i+1))
done

#!/bin/bash
# dW-kernel memory counters over tools/bench_update.py (one counter group per rocprofv3 pass, no
# trace domains): FETCH_SIZE (HBM/fabric reads), TCC hit/miss (L2), kernel trace for durations.
# usage: tools/pmc_dw.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/dwprof_$tag
mkdir -p $base/fetch $base/tcc
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $base/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/fetch/log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $base/tcc -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/tcc/log 2>&1 || exit $?
mkdir -p $base/write
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $base/write -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/write/log 2>&1 || exit $?

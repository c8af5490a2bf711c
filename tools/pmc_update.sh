#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes, no trace domains) over tools/bench_update.py.
# usage: tools/pmc_update.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/uprof_$tag
mkdir -p $base/trace $base/fetch $base/write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $base/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 10 > $base/trace/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $base/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/fetch/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $base/write -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/write/log 2>&1 || exit $?

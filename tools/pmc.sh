#!/bin/bash
# One rocprofv3 PMC pass (a single TCC counter group per pass; no trace domains) over a short
# bench run, from the repo root on the GPU box.
# usage: tools/pmc.sh <tag> <counter> [bench args...]
set -o pipefail
tag=$1; ctr=$2; shift 2
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_${tag}_${ctr}
mkdir -p $out
timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $out/bench.log 2>&1
rc=$?
echo "rocprof exit $rc" >> $out/bench.log
exit $rc

#!/bin/bash
# Kernel-trace + stats profile of a short bench run (run from the repo root on the GPU box).
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $out/bench.log 2>&1
rc=$?
echo "rocprof exit $rc" >> $out/bench.log
exit $rc

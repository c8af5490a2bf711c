#!/bin/bash
# rocprofv3 kernel-trace + stats of back-to-back sampler launches (tools/bench_sampler.py), then
# one PMC pass each for FETCH_SIZE and WRITE_SIZE (no trace domains with --pmc).
# usage: tools/profile_sampler.sh <tag>   SARGS='--envs 256 --config-dir ...' passes through to bench_sampler.py
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/sprof_$tag
mkdir -p $base/trace $base/fetch $base/write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $base/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_sampler.py --reps 200 $SARGS > $base/trace/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $base/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_sampler.py --reps 20 $SARGS > $base/fetch/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $base/write -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_sampler.py --reps 20 $SARGS > $base/write/log 2>&1 || exit $?

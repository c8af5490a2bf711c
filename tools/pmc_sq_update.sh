#!/bin/bash
# SQ counters (one pass, no trace domains) for the update kernels over tools/bench_update.py.
# usage: tools/pmc_sq_update.sh <tag> [DPPO_LIB path]
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/sqprof_$tag
mkdir -p $base
[ -n "$2" ] && export DPPO_LIB=$2
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $base -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 3 > $base/log 2>&1

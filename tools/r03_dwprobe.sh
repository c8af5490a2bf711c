#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 python -u tools/probe_dw_blas.py > gpurun_out/dwprobe.log 2>&1 || { tail -20 gpurun_out/dwprobe.log; exit 1; }
tail -1 gpurun_out/dwprobe.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bu -o run -- python3 -u tools/bench_update.py --reps 5 > gpurun_out/prof_bu.log 2>&1 || { tail -20 gpurun_out/prof_bu.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blas -o run -- python3 -u tools/probe_dw_blas.py --reps 5 > gpurun_out/prof_blas.log 2>&1 || { tail -20 gpurun_out/prof_blas.log; exit 1; }
echo done

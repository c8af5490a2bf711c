#!/bin/bash
# kernel timelines of tools/bench_update.py (fused minibatch) with DPPO_TAIL_OVERLAP=1 and 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  base=$GRAFT_REPO_ROOT/gpurun_out/tl_$v; mkdir -p $base
  DPPO_TAIL_OVERLAP=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $base -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 5 > $base/log 2>&1 || exit 1
  f=$(find $base -name 'run_kernel_trace.csv' | head -1)
  echo "== overlap=$v"; python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py $f 24
done

#!/bin/bash
# Round-6 closing evidence: the whole-iteration kernel trace of the headline workload (the bench's
# kernels.profile_crosscheck source) and the wrapper-stack env lines (C simulator; 0 / 20 us of emulated
# physics per env sub-step; 1 / 4 / 8 host threads). usage: tools/r06_end.sh <tag>
set -o pipefail
tag=${1:-r06end}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/profile.sh $tag --steps 3 --warmup 1 || { tail -20 gpurun_out/prof_$tag/bench.log; exit 1; }
tail -2 gpurun_out/prof_$tag/bench.log | cut -c1-200
for spec in "1 0" "4 0" "1 20" "8 20"; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --env lowdim --env-threads $1 --sim-cost-us $2 --no-cpu-baseline \
    > gpurun_out/bench_lowdim_t$1_c$2_$tag.log 2>&1 || { echo "lowdim bench failed"; tail -30 gpurun_out/bench_lowdim_t$1_c$2_$tag.log; exit 1; }
  tail -1 gpurun_out/bench_lowdim_t$1_c$2_$tag.log | cut -c1-160
done

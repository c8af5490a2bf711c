#!/bin/bash
# GPU tests + bench + sampler profile in one gpurun call (each step time-limited, chained).
# usage: tools/round_check.sh <tag>     LOWDIM=1 adds bench lines on the wrapper-stack env (1 and 4
# host threads, and 4 threads with 20 us of emulated physics per env sub-step); NOPROF=1 skips the
# sampler profile; TESTS=<pytest -k expr> narrows the GPU tests
set -o pipefail
tag=${1:-chk}
cd $GRAFT_REPO_ROOT
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTS:+-k "$TESTS"} > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
if [ -n "$LOWDIM" ]; then
  for spec in "1 0" "4 0" "1 20" "8 20"; do
    set -- $spec
    timeout -k 10 300 python -u bench.py --env lowdim --env-threads $1 --sim-cost-us $2 --no-cpu-baseline \
      > gpurun_out/bench_lowdim_t$1_c$2_$tag.log 2>&1 || { echo "lowdim bench failed"; tail -30 gpurun_out/bench_lowdim_t$1_c$2_$tag.log; exit 1; }
    tail -1 gpurun_out/bench_lowdim_t$1_c$2_$tag.log
  done
fi
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
[ -n "$NOPROF" ] || { bash tools/profile_sampler.sh $tag && echo profiled; }

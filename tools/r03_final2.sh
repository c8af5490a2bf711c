#!/bin/bash
# r03 round state (session 2): GPU tests, the default bench line (with its CPU baseline), smoke, the
# sampler's kernel-trace + PMC passes, an iteration kernel trace and the emulated W = 8 rank line
set -o pipefail
tag=${1:-r03x}
cd $GRAFT_REPO_ROOT
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-300
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
bash tools/profile_sampler.sh $tag || { echo "profile_sampler failed"; exit 1; }
bash tools/profile.sh $tag --steps 2 --warmup 1 || { echo "profile failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/update_timeline.py gpurun_out/prof_$tag/run_kernel_trace.csv 90 > gpurun_out/${tag}_update_timeline.txt || true
timeout -k 10 400 python -u bench.py --emulate-ranks 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_emu8_$tag.log 2>&1 || { echo "emu failed"; tail -20 gpurun_out/bench_emu8_$tag.log; exit 1; }
tail -1 gpurun_out/bench_emu8_$tag.log | cut -c1-300
echo done

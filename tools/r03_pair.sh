#!/bin/bash
# r03: the pair sampler vs the one-tile sampler (timing + bit identity), parity tests, a bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03c}
DPPO_SPLIT_PAIR=0 timeout -k 10 120 python -u tools/bench_sampler.py --tag single_$tag --reps 300 > gpurun_out/samp_single_$tag.log 2>&1 || { tail -20 gpurun_out/samp_single_$tag.log; exit 1; }
tail -1 gpurun_out/samp_single_$tag.log
timeout -k 10 120 python -u tools/bench_sampler.py --tag pair_$tag --reps 300 > gpurun_out/samp_pair_$tag.log 2>&1 || { tail -20 gpurun_out/samp_pair_$tag.log; exit 1; }
tail -1 gpurun_out/samp_pair_$tag.log
python -c "
import numpy as np; a=np.load('gpurun_out/sampler_single_$tag.npy'); b=np.load('gpurun_out/sampler_pair_$tag.npy')
print('bit-identical:', np.array_equal(a,b), 'max diff', float(np.abs(a-b).max()), 'finite', bool(np.isfinite(b).all()))"
timeout -k 10 800 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/r03_pair_tests_$tag.log 2>&1 || { tail -40 gpurun_out/r03_pair_tests_$tag.log; exit 1; }
tail -2 gpurun_out/r03_pair_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { tail -30 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log

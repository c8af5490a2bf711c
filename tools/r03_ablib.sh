#!/bin/bash
# r03: GPU tests, then same-box A/B of the working tree's library against a variant
# (tools/base_build.sh <tag>): isolated update (bench_update) and the bench, alternating
# usage: tools/r03_ablib.sh <tag> <variant>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; var=$2
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
for i in 1 2; do
  for lib in tree $var; do
    if [ $lib = tree ]; then unset DPPO_LIB; else export DPPO_LIB=$V/libdppo_hip_$lib.so; fi
    timeout -k 10 180 python -u tools/bench_update.py --reps 20 > gpurun_out/ab_bu_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/ab_bu_${lib}_$i.log; exit 1; }
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/ab_bench_${lib}_$i.log; exit 1; }
    python3 -c "
import json
u=json.loads(open('gpurun_out/ab_bu_${lib}_$i.log').read().strip().splitlines()[-1])
d=json.loads(open('gpurun_out/ab_bench_${lib}_$i.log').read().strip().splitlines()[-1])
print('$lib', 'iso_mb', round(u['minibatch_ms'],4), 'lp', round(u['logprob_pass_ms'],4), '| bench', round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4), 'roll', round(d['rollout_s_per_iter']*1e3,2))"
  done
done

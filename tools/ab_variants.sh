#!/bin/bash
# Sampler time per launch for the main library and lib/variants/libdppo_hip_<tag>.so, interleaved
# twice (bench workload: hopper, bf16, 64 envs). usage: tools/ab_variants.sh <tag>...
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    echo -n "$v "
    DPPO_LIB=$L timeout -k 5 60 python tools/bench_sampler.py --tag $v --reps 300 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
  done
done

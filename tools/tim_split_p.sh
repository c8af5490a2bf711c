#!/bin/bash
# Phase timers of the split sampler (timing build lib/variants/libdppo_hip_tim.so) for P = 4 and 8.
set -o pipefail
mkdir -p gpurun_out
L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_tim.so
for p in 4 8; do
  DPPO_LIB=$L DPPO_SPLIT_P=$p timeout -k 5 120 python tools/bench_sampler.py --tag tim_p$p > gpurun_out/tim_p$p.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/tim_p$p.json')); c=d['cycles_per_step']; w=c.pop('wg0_steps'); print('P=$p', round(d['ms_per_launch']*1e3,1), c); print('  wg0 step5', w[5])"
done

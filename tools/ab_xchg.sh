#!/bin/bash
# A/B of the split sampler's exchange form (auto = L2-local when a group shares one XCD, shared =
# always write-through): default build, then the phase-timer build. Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_tim.so
for mode in auto shared auto shared; do
  DPPO_SPLIT_XCHG=$mode timeout -k 5 120 python tools/bench_sampler.py --tag $mode --reps 300 | cut -c1-200 || exit 1
done
for mode in auto shared; do
  DPPO_LIB=$L DPPO_SPLIT_XCHG=$mode timeout -k 5 120 python tools/bench_sampler.py --tag tim_$mode > gpurun_out/ab_tim_$mode.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_tim_$mode.json')); c=d['cycles_per_step']; c.pop('wg0_steps'); print('$mode', d['ms_per_launch'], c)"
done

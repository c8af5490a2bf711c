#!/bin/bash
# the split sampler's l1 read-ahead depth (DPPO_S4_L1D: u1 fragment reads issued ahead of the MFMA
# chain) at 0 / 1 against the default, hopper bf16 64 envs and fp32, 300 launches each, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default l1d1 l1d0; do
    if [ $v = default ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    for p in bf16 fp32; do
      echo -n "$v $p "
      DPPO_LIB=$L timeout -k 5 90 python tools/bench_sampler.py --precision $p --tag $v --reps 300 \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
    done
  done
done

#!/bin/bash
# DPPO_S4_INREADY=0 (the in-Dense operands left to the compiler's schedule) against the default on the
# other shapes: walker2d 256 envs bf16, hopper fp32, hopper DDIM 512 fp16; 300 launches, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
F=$GRAFT_REPO_ROOT/cfg/gym/finetune
for rep in 1 2; do
  for v in default inr0; do
    if [ $v = default ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    for spec in "walker256 --envs 256 --config-dir $F/walker2d-v2 --config-name ft_ppo_diffusion_mlp" "fp32 --precision fp32" \
                "ddim512 --envs 512 --precision fp16 --config-dir $F/hopper-v2 --config-name ft_ppo_diffusion_mlp_ddim"; do
      set -- $spec; name=$1; shift
      echo -n "$v $name "
      DPPO_LIB=$L timeout -k 5 90 python tools/bench_sampler.py --reps 300 --tag $v "$@" \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
    done
  done
done

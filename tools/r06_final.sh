#!/bin/bash
# Round-6 end-of-round lines: the emulated W = 8 hopper rank and the other configs' shards (walker2d
# 256 envs, halfcheetah 256 as one rank of 8, hopper DDIM 512 fp16 as one rank of 8, hopper 64 fp32),
# then the sampler profiles (rocprofv3 stats + FETCH / WRITE) of hopper bf16, walker2d 256 and fp32.
# usage: tools/r06_final.sh <tag>
set -o pipefail
tag=${1:-r06g}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/bench_${tag}_emu8.log 2>&1 \
  || { tail -20 gpurun_out/bench_${tag}_emu8.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_emu8.log | cut -c1-300
ONLY="walker256|cheetah256_emu8|ddim512_emu8|hopper64_fp32" NOPROF=1 bash tools/r05_configs.sh $tag || exit 1
bash tools/profile_sampler.sh $tag || exit 1
echo prof hopper
SARGS="--envs 256 --config-dir $GRAFT_REPO_ROOT/cfg/gym/finetune/walker2d-v2 --config-name ft_ppo_diffusion_mlp" bash tools/profile_sampler.sh ${tag}_walker256 || exit 1
echo prof walker
SARGS="--precision fp32" bash tools/profile_sampler.sh ${tag}_fp32 || exit 1
echo prof fp32

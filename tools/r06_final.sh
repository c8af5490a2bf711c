#!/bin/bash
# Round-6 end-of-round lines: the emulated W = 8 hopper rank, the other configs' shards, and the fp32
# sampler A/B (8 members of 4 waves, the default, against 4 of 8: lib/variants/libdppo_hip_f32p4.so,
# tools/variant_build.sh f32p4 "-DDPPO_F32_P=4"). usage: tools/r06_final.sh <tag>
set -o pipefail
tag=${1:-r06g}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/bench_${tag}_emu8.log 2>&1 \
  || { tail -20 gpurun_out/bench_${tag}_emu8.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_emu8.log | cut -c1-300
ONLY="walker256|cheetah256_emu8|ddim512_emu8|hopper64_fp32" NOPROF=1 bash tools/r05_configs.sh $tag || exit 1
for rep in 1 2; do
  for v in default f32p4; do
    if [ $v = default ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    echo -n "fp32 sampler $v "
    DPPO_LIB=$L timeout -k 5 90 python tools/bench_sampler.py --precision fp32 --tag $v --reps 300 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
  done
done

#!/bin/bash
# Bench lines of the other BASELINE configs' per-GPU shards + their sampler profiles:
#   walker2d 256 envs bf16 (config 3), halfcheetah 256 envs bf16 as one rank of 8 (config 4's shard),
#   hopper DDIM 512 envs fp16 as one rank of 8 (config 5's shard), hopper 64 envs fp32 (config 2 at the
#   reference's precision). usage: tools/r05_configs.sh <tag>   NOPROF=1 skips the rocprof passes,
#   ONLY=<regex> runs the matching lines only
set -o pipefail
tag=${1:-cfg}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
F=cfg/gym/finetune
run() {   # name, bench args...
  local name=$1; shift
  [ -n "$ONLY" ] && [[ ! $name =~ $ONLY ]] && return 0
  timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${tag}_$name.log 2>&1 \
    || { echo "bench $name failed"; tail -30 gpurun_out/bench_${tag}_$name.log; exit 1; }
  python - gpurun_out/bench_${tag}_$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], round(d["value"]), "env-steps/s", "ms/it", round(d["ms_per_step"], 2), "roll", round(1e3 * d["rollout_s_per_iter"], 2),
      "upd", round(1e3 * d["update_s_per_iter"], 2), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4), "sampler_us",
      round(r["avg_launch_ms"] * 1e3, 2), "frac", round(r["frac"], 4), d["dtype"])
PY
}
run walker256 --config-dir $F/walker2d-v2 --config-name ft_ppo_diffusion_mlp --envs-per-gpu 256
run cheetah256_emu8 --config-dir $F/halfcheetah-v2 --config-name ft_ppo_diffusion_mlp --envs-per-gpu 256 --emulate-ranks 8
run ddim512_emu8 --config-dir $F/hopper-v2 --config-name ft_ppo_diffusion_mlp_ddim --envs-per-gpu 512 --emulate-ranks 8
run hopper64_fp32 --precision fp32
# the wrapper-stack env (C simulator, 0 or 20 us of emulated physics per env sub-step), 1/4/8 threads
run lowdim_t1_c0 --env lowdim --env-threads 1
run lowdim_t4_c0 --env lowdim --env-threads 4
run lowdim_t1_c20 --env lowdim --env-threads 1 --sim-cost-us 20
run lowdim_t8_c20 --env lowdim --env-threads 8 --sim-cost-us 20
[ -n "$NOPROF" ] && exit 0
SARGS="--envs 256 --config-dir $GRAFT_REPO_ROOT/$F/walker2d-v2 --config-name ft_ppo_diffusion_mlp" bash tools/profile_sampler.sh ${tag}_walker256 && echo prof walker
SARGS="--envs 512 --precision fp16 --config-dir $GRAFT_REPO_ROOT/$F/hopper-v2 --config-name ft_ppo_diffusion_mlp_ddim" bash tools/profile_sampler.sh ${tag}_ddim512 && echo prof ddim

#!/bin/bash
# the in-Dense state k-step in LDS for every KX = 2 shape: the sampler parity tests of walker2d /
# halfcheetah and fp32, the fp32 iteration seeds, and the launch times (walker2d 256 envs bf16,
# halfcheetah 256 bf16, hopper 64 fp32; 300 launches each)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_iteration_gpu.py -m gpu \
  -k "walker or cheetah or fp32 or config3 or config4 or test_iterations_match_oracle" > gpurun_out/sbl_tests.log 2>&1 \
  || { tail -30 gpurun_out/sbl_tests.log; exit 1; }
tail -1 gpurun_out/sbl_tests.log
F=$GRAFT_REPO_ROOT/cfg/gym/finetune
for rep in 1 2; do
  for spec in "walker256 --envs 256 --config-dir $F/walker2d-v2 --config-name ft_ppo_diffusion_mlp" \
              "cheetah256 --envs 256 --config-dir $F/halfcheetah-v2 --config-name ft_ppo_diffusion_mlp" \
              "fp32 --precision fp32"; do
    set -- $spec; name=$1; shift
    echo -n "$name "; timeout -k 5 90 python tools/bench_sampler.py --reps 300 "$@" \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
  done
done

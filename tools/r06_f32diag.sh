#!/bin/bash
# fp32 split sampler at 8 members: its own parity tests, the seed-44 iteration test under the 8- and
# 4-member builds (lib/variants/libdppo_hip_f32p4.so), and the sampler A/B (300 launches each)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -m gpu -k "fp32 and (sampler or split)" > gpurun_out/f32diag_kern.log 2>&1 || { tail -30 gpurun_out/f32diag_kern.log; exit 1; }
tail -2 gpurun_out/f32diag_kern.log
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_f32diag_p4.jsonl
DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_f32p4.so timeout -k 10 300 $T tests/test_iteration_gpu.py -m gpu -k "test_iterations_match_oracle and 44" > gpurun_out/f32diag_it_p4.log 2>&1; echo "p4 iteration rc $?"; tail -2 gpurun_out/f32diag_it_p4.log
for rep in 1 2; do
  for v in default f32p4; do
    if [ $v = default ]; then L=""; else L=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so; fi
    echo -n "fp32 sampler $v "
    DPPO_LIB=$L timeout -k 5 90 python tools/bench_sampler.py --precision fp32 --tag $v --reps 300 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
  done
done

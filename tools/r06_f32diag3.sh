#!/bin/bash
# fp32 8-member sampler with the state pre-projection: its parity tests, its time per launch, the
# seed-44 iteration numbers, and the float64 oracle's own sensitivity at that seed
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -m gpu -k "fp32 and (sampler or split)" > gpurun_out/f32diag3_kern.log 2>&1 || { tail -30 gpurun_out/f32diag3_kern.log; exit 1; }
tail -1 gpurun_out/f32diag3_kern.log
for rep in 1 2; do
  echo -n "fp32 sampler "; timeout -k 5 90 python tools/bench_sampler.py --precision fp32 --reps 300 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_launch']*1e3,2), 'us')" || exit 1
done
timeout -k 10 300 python -u tools/iter_parity_probe.py 44 > gpurun_out/probe44_sb.log 2>&1 || { tail -20 gpurun_out/probe44_sb.log; exit 1; }
grep '^{' gpurun_out/probe44_sb.log
timeout -k 10 600 python -u tools/oracle_sensitivity.py 44 --trials 3 > gpurun_out/oracle_sens44.log 2>&1 || { tail -20 gpurun_out/oracle_sens44.log; exit 1; }
grep '^{' gpurun_out/oracle_sens44.log

#!/bin/bash
# r03: the critic gate: its equivalence test, isolated fused-minibatch A/B, kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "critic_gate or full_size or minibatch_grads" > gpurun_out/gate_tests.log 2>&1 || { tail -40 gpurun_out/gate_tests.log; exit 1; }
tail -1 gpurun_out/gate_tests.log
for i in 1 2; do for v in 1 0; do DPPO_CRITIC_GATE=$v timeout -k 10 200 python tools/bench_update.py --reps 30 > gpurun_out/bu_gate_$v.log 2>&1 || exit 1; echo "gate=$v $(tail -1 gpurun_out/bu_gate_$v.log | cut -c1-120)"; done; done
cd /tmp && export TMPDIR=/tmp
base=$GRAFT_REPO_ROOT/gpurun_out/tlg_1; mkdir -p $base
DPPO_CRITIC_GATE=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $base -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_update.py --reps 5 > $base/log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh DPPO_CRITIC_GATE "1 0" 2

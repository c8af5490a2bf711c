#!/bin/bash
# r03: the critic's dW held until the actor's dW is done (parts 6 / 7): GPU tests, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_latecdw.log 2>&1 || { tail -40 gpurun_out/gpu_tests_latecdw.log; exit 1; }
tail -1 gpurun_out/gpu_tests_latecdw.log
bash tools/ab_env.sh DPPO_LATE_CRITIC_DW "1 0" 3

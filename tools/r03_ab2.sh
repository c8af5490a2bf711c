#!/bin/bash
# r03: GPU tests, then same-box A/B of an env knob on the bench (tools/ab_env.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; var=$2; vals=$3
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
bash tools/ab_env.sh $var "$vals" 2

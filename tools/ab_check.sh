#!/bin/bash
# A kernel change's GPU check in one gpurun call: the GPU tests selected by -k <expr>, then the
# sampler A/B of the working tree against lib/variants/libdppo_hip_<tag>.so (tools/base_build.sh).
# usage: tools/ab_check.sh <pytest -k expr> <variant tag>...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
k=$1; shift
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$k" > gpurun_out/abc_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/abc_tests.log; exit 1; }
tail -3 gpurun_out/abc_tests.log
bash tools/ab_variants.sh "$@" > gpurun_out/abc_ab.log 2>&1 || { echo "ab failed"; cat gpurun_out/abc_ab.log; exit 1; }
cat gpurun_out/abc_ab.log

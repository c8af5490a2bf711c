#!/bin/bash
# Round-5 counter evidence: the update kernels' SQ pass and FETCH / WRITE passes
# (tools/bench_update.py, 50,000-row minibatch) and the 64-env sampler's trace + FETCH / WRITE passes,
# each pass its own rocprofv3 run with a time limit. usage: tools/r05_pmc.sh <tag>   (DPPO_LIB passes through)
set -o pipefail
tag=${1:-pmc}
cd $GRAFT_REPO_ROOT
bash tools/pmc_sq_update.sh $tag && echo "sq ok" || { echo "sq pass failed"; exit 1; }
bash tools/pmc_update.sh $tag && echo "update fetch/write ok" || { echo "update passes failed"; exit 1; }
bash tools/profile_sampler.sh ${tag}_s64 && echo "sampler ok" || { echo "sampler passes failed"; exit 1; }

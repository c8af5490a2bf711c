#!/bin/bash
# Round-5 final check: the time-MLP backward's phases (timing build), then tests + bench + lowdim +
# smoke + sampler profile (round_check.sh), the emulated W = 8 rank's bench line and an iteration trace.
# usage: tools/r05_final.sh <tag>
set -o pipefail
tag=${1:-r05end}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rows in 50000 6250; do
  DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_tbtim2.so timeout -k 10 200 python -u tools/bench_update.py --reps 5 --rows $rows \
    > gpurun_out/tb_tbtim2_$rows.txt 2>&1 || { tail -20 gpurun_out/tb_tbtim2_$rows.txt; exit 1; }
  echo "tbtim2 $rows $(tail -1 gpurun_out/tb_tbtim2_$rows.txt)"
done
LOWDIM=1 bash tools/round_check.sh $tag || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/bench_${tag}_emu8.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_emu8.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_emu8.log | cut -c1-300
timeout -k 10 300 bash tools/profile.sh $tag

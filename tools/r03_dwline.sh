#!/bin/bash
# r03: dW stage size A/B (DPPO_DW_LINE 128 default vs 64) on the isolated update (bench_update) and
# the bench, same box
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
for i in 1 2; do
  for lib in default dwl64; do
    if [ $lib = default ]; then unset DPPO_LIB; else export DPPO_LIB=$V/libdppo_hip_$lib.so; fi
    timeout -k 10 180 python -u tools/bench_update.py --reps 20 > gpurun_out/dwl_bu_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/dwl_bu_${lib}_$i.log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/dwl_bu_${lib}_$i.log | cut -c1-120)"
  done
done
unset DPPO_LIB
cd /tmp && export TMPDIR=/tmp
for lib in default dwl64; do
  if [ $lib = default ]; then unset DPPO_LIB; else export DPPO_LIB=$V/libdppo_hip_$lib.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dwl_$lib -o run -- python3 -u $GRAFT_REPO_ROOT/tools/bench_update.py --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/dwl_prof_$lib.log 2>&1 || exit 1
done
echo done

#!/bin/bash
# r03: sampler launch time with one barrier of the folded step dropped (timing probes, wrong
# actions), against the default, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants
for i in 1 2; do
  for lib in default ns1 ns2 ns3; do
    if [ $lib = default ]; then unset DPPO_LIB; else export DPPO_LIB=$V/libdppo_hip_$lib.so; fi
    timeout -k 10 120 python -u tools/bench_sampler.py --reps 300 --tag $lib > gpurun_out/ns_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/ns_${lib}_$i.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/ns_${lib}_$i.log').read().strip().splitlines()[-1])
print('$lib', round(d['ms_per_launch']*1e3,2))"
  done
done

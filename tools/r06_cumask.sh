#!/bin/bash
# critic side stream on a CU subset (tools/cu_mask_probe.py): N = 1 and the emulated W = 8 rank
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cu_mask_probe.py --emulate-ranks 8 --iters 2 > gpurun_out/cumask_emu8.log 2>&1 || { tail -20 gpurun_out/cumask_emu8.log; exit 1; }
grep '^{' gpurun_out/cumask_emu8.log
timeout -k 10 400 python -u tools/cu_mask_probe.py --iters 3 > gpurun_out/cumask_n1.log 2>&1 || { tail -20 gpurun_out/cumask_n1.log; exit 1; }
grep '^{' gpurun_out/cumask_n1.log

#!/bin/bash
# The IPC all-reduce's tests and its per-call latency at the update's bucket sizes (0.54 MB, 2.2 MB)
# with W = 2 and 4 processes sharing cuda:0 (same-device IPC; not an xGMI figure).
# usage: tools/r06_ipc.sh <tag>
set -o pipefail
tag=${1:-r06ipc}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export DPPO_SINGLE_DEVICE=1
timeout -k 10 600 python -u -m pytest tests/test_collective_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for w in 2 4; do
  DPPO_IPC_OUT=gpurun_out/${tag}_latency_w$w.json timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29600 + w)) tools/ipc_latency.py \
    > gpurun_out/${tag}_latency_w$w.log 2>&1 || { tail -30 gpurun_out/${tag}_latency_w$w.log; exit 1; }
  cat gpurun_out/${tag}_latency_w$w.json
done

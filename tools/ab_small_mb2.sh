#!/bin/bash
# 6,250-row minibatches in the fused (data-parallel) update mode: dW split-K chunk counts.
set -o pipefail
mkdir -p gpurun_out
run() { echo -n "$1: "; env DPPO_SPLIT_UPDATE=0 $2 timeout -k 5 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch-size 6250 > gpurun_out/abs.log 2>&1 || { tail -5 gpurun_out/abs.log; exit 1; }; tail -1 gpurun_out/abs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f update %.2f ms mb %.3f ms' % (d['value'], d['update_s_per_iter']*1e3, d['ppo_minibatch_avg_ms']))"; }
run default "X=1"
run ch2 "DPPO_DW_CHUNKS=2"
run ch4 "DPPO_DW_CHUNKS=4"
run ch8 "DPPO_DW_CHUNKS=8"
run tk128 "DPPO_DW_TK=128"

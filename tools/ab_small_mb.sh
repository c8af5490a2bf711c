#!/bin/bash
# Update time at the per-rank minibatch of an 8-GPU run under the reference's global minibatch
# (50,000 / 8 = 6,250 rows; 51 minibatches per epoch): actor row-tile shapes.
set -o pipefail
mkdir -p gpurun_out
run() { echo -n "$1: "; env $2 timeout -k 5 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch-size 6250 > gpurun_out/abs.log 2>&1 || { tail -5 gpurun_out/abs.log; exit 1; }; tail -1 gpurun_out/abs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.0f update %.2f ms mb %.3f ms updates/s %.0f' % (d['value'], d['update_s_per_iter']*1e3, d['ppo_minibatch_avg_ms'], d['ppo_updates_per_sec']))"; }
run default "X=1"
run a32x8 "DPPO_ROWTILE=32x8"
run a32x8o4 "DPPO_ROWTILE=32x8o4"
run nosplit "DPPO_SPLIT_UPDATE=0"

#!/bin/bash
# update knobs on the emulated W = 8 rank (6,250-row minibatches), same box: tools/emu_knobs.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  env $2 timeout -k 10 200 python -u bench.py --emulate-ranks 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/emuk_$1.log 2>&1 || { tail -20 gpurun_out/emuk_$1.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/emuk_$1.log').read().strip().splitlines()[-1]); print('$1', round(d['value']), 'upd', round(d['update_s_per_iter']*1e3,2), 'mb', round(d['ppo_minibatch_avg_ms'],4))"
}
run base X=1
run tk128 DPPO_DW_TK=128
run ch64 DPPO_DW_CHUNKS=64
run ch128 DPPO_DW_CHUNKS=128
run ch512 DPPO_DW_CHUNKS=512
run zero64 DPPO_ZERO_BLOCKS=64
run zero4 DPPO_ZERO_BLOCKS=4
run base2 X=1

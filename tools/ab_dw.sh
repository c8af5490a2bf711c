#!/bin/bash
# A/B of the dW k-tile edge (DPPO_DW_TK = 128 / 256) on tools/bench_update.py, alternating.
set -o pipefail
for tk in 128 256 128 256; do
  DPPO_DW_TK=$tk timeout -k 5 120 python tools/bench_update.py --reps 30 | sed "s/^/tk=$tk /" | cut -c1-160 || exit 1
done

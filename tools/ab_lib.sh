#!/bin/bash
# A/B of two library builds on tools/bench_update.py, alternating (DPPO_LIB selects the build).
# usage: tools/ab_lib.sh <libA.so> <libB.so> [reps]
set -o pipefail
a=$1; b=$2; reps=${3:-30}
for lib in $a $b $a $b; do
  DPPO_LIB=$lib timeout -k 5 120 python tools/bench_update.py --reps $reps | sed "s|^|$(basename $lib) |" | cut -c1-200 || exit 1
done

#!/bin/bash
# Same-box A/B of an env knob on the N = 1 bench line and the emulated W = 8 rank's line.
# usage: tools/r06_ab.sh <tag> "<A env>" "<B env>" [pairs]    TESTS=<pytest -k expr> runs those GPU tests
# first; TRACE=1 adds the emulated rank's kernel trace under the B env; CFG="<bench args>" adds a third
# line per side with those bench arguments (e.g. a side config)
set -o pipefail
tag=$1; A=$2; B=$3; pairs=${4:-2}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" \
    > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
line() {   # label, env, bench args...
  local lab=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_$lab.log 2>&1 || { tail -20 gpurun_out/${tag}_$lab.log; exit 1; }
  python - gpurun_out/${tag}_$lab.log $lab <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), "ms/it", round(d["ms_per_step"], 2), "roll", round(1e3 * d["rollout_s_per_iter"], 2),
      "upd", round(1e3 * d["update_s_per_iter"], 2), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4), flush=True)
PY
}
for p in $(seq 1 $pairs); do
  for side in A B; do
    envs=$A; [ $side = B ] && envs=$B
    line ${side}${p}_n1 "$envs" || exit 1
    line ${side}${p}_emu8 "$envs" --emulate-ranks 8 || exit 1
    if [ -n "$CFG" ]; then line ${side}${p}_cfg "$envs" $CFG || exit 1; fi
  done
done
if [ -n "$TRACE" ]; then
  timeout -k 10 700 bash tools/emu_trace.sh $tag $B || exit 1
  head -45 gpurun_out/prof_emu_$tag/timeline.txt
fi

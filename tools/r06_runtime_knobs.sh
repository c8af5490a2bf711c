#!/bin/bash
# the rollout's runtime settings against their defaults (2 launch streams, a log-prob pass every 10 env
# steps): 3 / 4 streams, pass chunks of 5 / 20 / 40 (r06o: streams and chunk alone; r06p: combined;
# r06q: the best pair against its parts, three rounds); agent bench at N = 1
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/rk_$name.log 2>&1 || { tail -20 gpurun_out/rk_$name.log; exit 1; }
  python - gpurun_out/rk_$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), "roll_ms", round(1e3 * d["rollout_s_per_iter"], 2), "upd_ms", round(1e3 * d["update_s_per_iter"], 2))
PY
}
for r in 1 2 3; do
  run default DPPO_X=0
  run s4c20 DPPO_ROLLOUT_STREAMS=4 DPPO_PASS_CHUNK=20
  run s4 DPPO_ROLLOUT_STREAMS=4
  run c20 DPPO_PASS_CHUNK=20
done

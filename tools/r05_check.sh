#!/bin/bash
# Round 5 check: GPU tests, then the bench (N = 1 and one emulated W = 8 rank) with the one-launch
# actor step (default) and the r04 step (DPPO_FUSED_STEP=critic) alternating, each step time-limited.
# usage: tools/r05_check.sh <tag>   TESTS=<pytest -k expr> narrows the tests; NOTESTS=1 skips them;
# PAIRS=<n> A/B rounds (default 1); NOBENCH=1 skips the bench A/B; AB_VAR / AB_VALS: the knob and its
# values (default DPPO_FUSED_STEP, "all critic")
set -o pipefail
tag=${1:-chk}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DPPO_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_$tag.jsonl
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTS:+-k "$TESTS"} \
    > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
  tail -3 gpurun_out/gpu_tests_$tag.log
fi
# VARTESTS="<tag>..." runs the sampler parity tests against lib/variants/libdppo_hip_<tag>.so
for v in $VARTESTS; do
  DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -v \
    --timeout 120 --timeout-method thread -k "sampler or pipelined" > gpurun_out/gpu_tests_${tag}_$v.log 2>&1 \
    || { echo "variant $v tests failed"; tail -40 gpurun_out/gpu_tests_${tag}_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/gpu_tests_${tag}_$v.log)"
done
[ -n "$NOBENCH" ] && { [ -n "$VARIANTS" ] && bash tools/ab_variants.sh $VARIANTS; exit 0; }
for r in $(seq 1 ${PAIRS:-1}); do
  for mode in ${AB_VALS:-all critic}; do
    env ${AB_VAR:-DPPO_FUSED_STEP}=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${tag}_${mode}_$r.log 2>&1 \
      || { echo "bench failed"; tail -30 gpurun_out/bench_${tag}_${mode}_$r.log; exit 1; }
    python - gpurun_out/bench_${tag}_${mode}_$r.log $mode <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "N=1", round(d["value"]), "ms/it", round(d["ms_per_step"], 2), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4),
      "roll_ms", round(1e3 * d["rollout_s_per_iter"], 2), "upd_ms", round(1e3 * d["update_s_per_iter"], 2))
PY
    env ${AB_VAR:-DPPO_FUSED_STEP}=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline --emulate-ranks 8 > gpurun_out/bench_${tag}_emu8_${mode}_$r.log 2>&1 \
      || { echo "emu bench failed"; tail -30 gpurun_out/bench_${tag}_emu8_${mode}_$r.log; exit 1; }
    python - gpurun_out/bench_${tag}_emu8_${mode}_$r.log $mode <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "emu8", round(d["value"]), "ms/it", round(d["ms_per_step"], 2), "mb_ms", round(d["ppo_minibatch_avg_ms"], 4),
      "roll_ms", round(1e3 * d["rollout_s_per_iter"], 2), "upd_ms", round(1e3 * d["update_s_per_iter"], 2))
PY
  done
done
[ -n "$VARIANTS" ] && bash tools/ab_variants.sh $VARIANTS
exit 0

# usage: tools/_uvariants.sh tag1 tag2 ...  (update minibatch timing: default lib vs lib/variants/libdppo_hip_<tag>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu.log 2>&1 || { tail -20 gpurun_out/bu.log; exit 1; }
  echo default $(tail -1 gpurun_out/bu.log | cut -c1-120)
  for t in "$@"; do
    DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$t.so timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu_$t.log 2>&1 || { tail -20 gpurun_out/bu_$t.log; exit 1; }
    echo $t $(tail -1 gpurun_out/bu_$t.log | cut -c1-120)
  done
done

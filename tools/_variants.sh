# usage: tools/_variants.sh tag1 tag2 ...   (default lib + lib/variants/libdppo_hip_<tag>.so, sampler only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_sampler.py > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
  tail -1 gpurun_out/bs.log | cut -c1-100
  for t in "$@"; do
    DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$t.so timeout -k 10 120 python -u tools/bench_sampler.py --tag $t > gpurun_out/bs_$t.log 2>&1 || { tail -20 gpurun_out/bs_$t.log; exit 1; }
    tail -1 gpurun_out/bs_$t.log | cut -c1-100
  done
done

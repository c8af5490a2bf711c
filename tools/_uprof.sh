set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu_plain.log 2>&1 || { tail -20 gpurun_out/bu_plain.log; exit 1; }
tail -1 gpurun_out/bu_plain.log
DPPO_LIB=$GRAFT_REPO_ROOT/diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_rtime.so timeout -k 10 120 python -u tools/bench_update.py > gpurun_out/bu_rtime.log 2>&1 || { tail -20 gpurun_out/bu_rtime.log; exit 1; }
tail -1 gpurun_out/bu_rtime.log
bash tools/pmc_update.sh $1 && echo pmc-ok

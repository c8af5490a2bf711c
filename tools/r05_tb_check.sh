set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r05z.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r05z.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r05z.log
for v in tbtim tbold; do
  for rows in 50000 6250; do
    DPPO_LIB=diffusionpolicyoptimization_amd/lib/variants/libdppo_hip_$v.so timeout -k 10 200 python -u tools/bench_update.py --reps 5 --rows $rows > gpurun_out/tb_${v}_$rows.txt 2>&1 || { tail -20 gpurun_out/tb_${v}_$rows.txt; exit 1; }
    echo "$v $rows $(tail -1 gpurun_out/tb_${v}_$rows.txt)"
  done
done
bash tools/ab_bench_lib.sh pairs 2

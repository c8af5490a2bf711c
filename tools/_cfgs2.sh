set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 1 --config-dir cfg/gym/finetune/walker2d-v2 --config-name ft_ppo_diffusion_mlp --envs-per-gpu 256 > gpurun_out/b_walker.log 2>&1 || { tail -5 gpurun_out/b_walker.log; exit 1; }
tail -1 gpurun_out/b_walker.log

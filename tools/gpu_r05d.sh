set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_shapes.py tests/test_gpu_step.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05d_t1.log 2>&1 || { echo T1FAIL; tail -30 gpurun_out/r05d_t1.log; exit 1; }
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-report gpurun_out/r05d_k.json > gpurun_out/r05d_bench.log 2>&1
tail -1 gpurun_out/r05d_t1.log
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05d_bench.log

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_williamson.py tests/test_gpu_jw06.py tests/test_gpu_damping.py tests/test_gpu_step.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1
echo rc=$? >> gpurun_out/r05b_tests.log
for m in 1 0; do
  GTFV3_THERMO_SPLIT=$m timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-report gpurun_out/r05b_k_split$m.json > gpurun_out/r05b_bench_split$m.log 2>&1 || exit 1
done
tail -2 gpurun_out/r05b_tests.log
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05b_bench_split*.log

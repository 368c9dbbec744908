set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-report gpurun_out/r05h_kernels.json > gpurun_out/r05h_bench.json 2>gpurun_out/r05h_bench.err || exit 1
for p in 8 6; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --rank-proxy $p > gpurun_out/r05h_proxy$p.json 2>gpurun_out/r05h_proxy$p.err || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05h_*.json

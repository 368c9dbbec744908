set -o pipefail
cd $GRAFT_REPO_ROOT
for sp in 58 0; do
  GTFV3_TP_SPANS=$sp timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-report gpurun_out/r05f_k$sp.json > gpurun_out/r05f_b$sp.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05f_b*.log

set -o pipefail
cd $GRAFT_REPO_ROOT
for lv in 1 2 4; do
  GTFV3_TP_EXLV=$lv timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-report gpurun_out/r05e_k$lv.json > gpurun_out/r05e_b$lv.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05e_b*.log

#!/bin/bash
# A/B of environment settings on one box: bench.py (no CPU baseline, no kernel timing) for each
# setting in turn, twice, so box-to-box spread drops out of the comparison.
#   usage: tools/ab_bench.sh TAG "ENV_A" "ENV_B" [...]   (each ENV a space-separated VAR=value list, or "-")
#   extra bench args via BENCH_ARGS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tag=$1; shift
for rep in 1 2; do
  n=0
  for envs in "$@"; do
    n=$((n + 1))
    [ "$envs" = "-" ] && envs=""
    out=gpurun_out/${tag}_${n}_${rep}.json
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 20 $BENCH_ARGS > "$out" 2> "$out.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('$tag', '$n', '$envs', 'rep $rep', round(d['ms_per_step'], 3), round(d['step_times']['min_ms'], 3))"
  done
done

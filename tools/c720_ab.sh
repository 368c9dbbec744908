#!/bin/bash
# C720 L137 x 54 tracers, the 8-rank share (rank 0 of 8, null transport): A/B of env settings
#   usage: tools/c720_ab.sh TAG "ENV_A" "ENV_B" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tag=$1; shift
n=0
for envs in "$@"; do
  n=$((n + 1))
  [ "$envs" = "-" ] && envs=""
  out=gpurun_out/${tag}_${n}.json
  env $envs timeout -k 10 400 python3 bench.py --npx 721 --npz 137 --nq 54 --rank-proxy 8 --steps 3 --warmup 1 \
    --no-cpu-baseline --kernel-report gpurun_out/${tag}_${n}_kernels.json > "$out" 2> "$out.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); k=json.load(open('gpurun_out/${tag}_${n}_kernels.json')); r=[v['ms_per_step'] for kk,v in k.items() if 'remap_blkq' in kk]; print('$tag', '$n', '$envs', round(d['ms_per_step'], 2), 'remap_blkq', r)"
done

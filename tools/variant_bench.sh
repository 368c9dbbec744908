#!/bin/bash
# Build and bench source variants of one csrc file on the GPU box:
#   tools/variant_bench.sh <csrc file name> <variant file>...
# Each variant replaces csrc/<file>, rebuilds, runs a short bench with the
# per-kernel report into gpurun_out/kern_<variant>.json.  The file is restored after.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
target=geosongpu-ci_amd/csrc/$1; shift
cp "$target" /tmp/variant_orig
for v in "$@"; do
  name=$(basename "$v" .hip)
  cp "$v" "$target"
  make -C geosongpu-ci_amd/csrc -j16 > gpurun_out/build_$name.log 2>&1 || { echo "build $name failed"; continue; }
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      --kernel-report gpurun_out/kern_$name.json > gpurun_out/bench_$name.log 2>&1
  rc=$?
  echo "variant $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$name.log)"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && break
done
cp /tmp/variant_orig "$target"
make -C geosongpu-ci_amd/csrc -j16 > /dev/null 2>&1

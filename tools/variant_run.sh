#!/bin/bash
# tools/variant_run.sh <csrc file> "<command>" <variant>...: for each variant file, swap it
# in, rebuild and run the command (output gpurun_out/var_<variant>.log); restores the file.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
target=geosongpu-ci_amd/csrc/$1; cmd=$2; shift 2
cp "$target" /tmp/variant_orig
for v in "$@"; do
  name=$(basename "$v" .hip)
  cp "$v" "$target"
  make -C geosongpu-ci_amd/csrc -j16 > gpurun_out/build_$name.log 2>&1 || { echo "build $name failed"; continue; }
  timeout -k 10 300 bash -c "$cmd" > gpurun_out/var_$name.log 2>&1
  rc=$?
  echo "variant $name rc=$rc"; tail -n 8 gpurun_out/var_$name.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && break
done
cp /tmp/variant_orig "$target"
make -C geosongpu-ci_amd/csrc -j16 > /dev/null 2>&1

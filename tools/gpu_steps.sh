#!/bin/bash
# Run GPU steps in order on the gpurun box; each step under its own time limit.
# A step that fails with an ordinary error (exit 1: failed tests / Python exception)
# lets the next step run; any fault-like exit (abort, segfault, time limit, ...) ends
# the script at once so nothing more touches the GPU after a fault.
#   usage: tools/gpu_steps.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
final=0
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc time=$(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    final=$rc
    if [ $rc -ne 1 ]; then echo "stopping after fault-like exit $rc"; exit $rc; fi
  fi
done
exit $final

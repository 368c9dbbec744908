#!/bin/bash
# Decomposition-invariance probe: the 1x1 vs 2x2 step test under each riem / remap form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rv in 0 1; do for mv in 0 2 1; do
  echo "== GTFV3_RIEM=$rv GTFV3_REMAP=$mv"
  GTFV3_RIEM=$rv GTFV3_REMAP=$mv timeout -k 10 120 python -u -m pytest -q -x --timeout 100 --timeout-method thread \
    tests/test_gpu_step.py -k decomposition_invariant 2>&1 | tail -3 || { rc=$?; [ $rc -ne 1 ] && exit $rc; }
done; done
exit 0

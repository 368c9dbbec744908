set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05g_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r05g_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r05g

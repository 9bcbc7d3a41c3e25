set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab3_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/libab.sh lib_base default lib_base default

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_codecs_fast.py tests/test_gpu_codecs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codecs_fast.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/codecs_fast.log
exit $rc

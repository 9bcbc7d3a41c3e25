set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c3.log; tail -1 gpurun_out/bench_c4.log

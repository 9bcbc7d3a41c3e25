set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -30 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench1.log 2>&1
echo "bench rc=$?"; cat gpurun_out/bench1.log

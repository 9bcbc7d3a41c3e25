# One GPU iteration on the in-tree build: the GPU test suite, then the default bench line
# (what the driver runs), each under its own time limit; stops at the first failure.
# usage: bash tools/gpu_step.sh [pytest -k expression]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc

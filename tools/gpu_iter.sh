# One build -> measure iteration on the GPU box: GPU tests, a short bench, a kernel-trace profile.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-iter}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"
cut -d, -f1-4 gpurun_out/prof_${TAG}/run_kernel_stats.csv | cut -c1-160 | head -8

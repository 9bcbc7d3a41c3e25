# The section-4b codec tests, then their kernel times (tools/codecs_bench.py under rocprofv3
# --kernel-trace --stats, at 2^26 and 2^28 Independent symbols), each under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_codecs.py > gpurun_out/codecs_tests.log 2>&1
rc=$?; echo "codecs tests rc=$rc"; tail -2 gpurun_out/codecs_tests.log; [ $rc -eq 0 ] || exit $rc
for sz in "26 24" "28 26"; do
  set -- $sz
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_codecs_$1 -o run --output-format csv -- python3 tools/codecs_bench.py $1 $2 > gpurun_out/prof_codecs_$1.log 2>&1
  rc=$?; echo "codecs $1 rc=$rc"; grep "^{" gpurun_out/prof_codecs_$1.log; [ $rc -eq 0 ] || exit $rc
done

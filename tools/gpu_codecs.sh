# The section-4b codecs on the GPU: their parity tests, then tools/codecs_bench.py on the fast
# kernels (under rocprofv3 --kernel-trace --stats) and on the exact ones (ANS_CODECS_EXACT=1),
# each step under its own limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_codecs_fast.py tests/test_gpu_codecs.py > gpurun_out/codecs_tests.log 2>&1
rc=$?; echo "codecs tests rc=$rc"; tail -2 gpurun_out/codecs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_codecs -o run --output-format csv -- python3 tools/codecs_bench.py 28 26 > gpurun_out/codecs_fast.json 2> gpurun_out/codecs_fast.err
rc=$?; echo "fast rc=$rc"; cat gpurun_out/codecs_fast.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/codecs_fast.err; exit $rc; }
ANS_CODECS_EXACT=1 timeout -k 10 400 python3 tools/codecs_bench.py 28 26 > gpurun_out/codecs_exact.json 2> gpurun_out/codecs_exact.err
rc=$?; echo "exact rc=$rc"; cat gpurun_out/codecs_exact.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/codecs_exact.err; exit $rc; }

# Same-box A/B of the current build against lib_base: the parity tests named in AB_TESTS first
# (default: the C3/C4 parity and norm-range suites), then tools/inproc_ab.py in both orders with
# the caller's AB_CONFIG / AB_LOG2N.   usage: AB_CONFIG=c4 AB_LOG2N=29 bash tools/gpu_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-ab}
TESTS=${AB_TESTS:-tests/test_gpu_parity.py tests/test_gpu_norm_ranges.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/inproc_ab.py lib_base lib ${ITERS:-30} > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/inproc_ab.py lib lib_base ${ITERS:-30} > gpurun_out/${TAG}_ab_rev.txt 2>&1
rc=$?; echo "ab rev rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_ab_rev.txt | tail -6

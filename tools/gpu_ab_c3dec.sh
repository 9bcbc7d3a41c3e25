# C3 decoder A/B (r06 sign-bit symbol select): parity tests of the u-domain decoder, then the
# same-box in-process A/B against lib_base.   usage: bash tools/gpu_ab_c3dec.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-c3dec}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_norm_ranges.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/inproc_ab.py lib_base lib ${ITERS:-30} > gpurun_out/${TAG}_ab_c3.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c3.txt | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/inproc_ab.py lib lib_base ${ITERS:-30} > gpurun_out/${TAG}_ab_c3_rev.txt 2>&1
rc=$?; echo "ab rev rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_ab_c3_rev.txt | tail -6

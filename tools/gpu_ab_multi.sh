# Same-box A/B of the current build against lib_base on several configs: the parity tests in
# AB_TESTS first, then tools/inproc_ab.py in both orders per config ("c3" = the default C3 run,
# else AB_CONFIG=<cfg> with AB_LOG2N from cfg:log2n).
#   usage: bash tools/gpu_ab_multi.sh <tag> c3 c4:29 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
TESTS=${AB_TESTS:-tests/test_gpu_parity.py tests/test_gpu_norm_ranges.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "$@"; do
  name=${cfg%%:*}; n=${cfg#*:}
  if [ "$name" = c3 ]; then unset AB_CONFIG AB_LOG2N; else export AB_CONFIG=$name; [ "$n" != "$cfg" ] && export AB_LOG2N=$n; fi
  for order in "lib_base lib" "lib lib_base"; do
    timeout -k 10 300 python -u tools/inproc_ab.py $order ${ITERS:-30} > gpurun_out/${TAG}_ab_${name}.txt 2>&1
    rc=$?; echo "== $name ($order) rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_ab_${name}.txt | tail -3; [ $rc -eq 0 ] || exit $rc
  done
done

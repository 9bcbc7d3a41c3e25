# Selected GPU tests on the in-tree library, then same-box A/Bs (tools/inproc_ab.py).
# usage: bash tools/gpu_ab_multi.sh "<pytest -k expr>" "<config>:<libA>:<libB>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
K=$1; shift
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  IFS=: read cfg A B <<< "$spec"
  AB_CONFIG=$cfg timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-30} > gpurun_out/ab_${cfg}_$B.txt 2>&1
  rc=$?; echo "ab $cfg $A vs $B rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_${cfg}_$B.txt; [ $rc -eq 0 ] || exit $rc
done

# Same-box A/B of library builds on C3 only (tools/inproc_ab.py), each pair under its own limit.
# usage: bash tools/gpu_ab_c3.sh <libdir A> <libdir B> [<libdir C> ...]   (B, C, ... each against A)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
A=$1; shift
for B in "$@"; do
  AB_CONFIG=${AB_CONFIG:-c3} timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-40} > gpurun_out/ab_c3_$B.txt 2>&1
  rc=$?; echo "ab ${AB_CONFIG:-c3} $A vs $B rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_c3_$B.txt
  [ $rc -eq 0 ] || exit $rc
done

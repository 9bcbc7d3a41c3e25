# Same-box A/B of library builds on C4 only (tools/inproc_ab.py), each pair under its own limit.
# usage: bash tools/gpu_ab_c4.sh <libdir A> <libdir B> [<libdir C> ...]   (B, C, ... each against A)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
A=$1; shift
for B in "$@"; do
  AB_CONFIG=c4 timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-20} > gpurun_out/ab_c4_$B.txt 2>&1
  rc=$?; echo "ab c4 $A vs $B rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_c4_$B.txt
  [ $rc -eq 0 ] || exit $rc
done

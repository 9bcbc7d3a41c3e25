# Same-box A/B of library builds on C3 only (tools/inproc_ab.py), each pair run once per lib pair.
# usage: bash tools/gpu_ab_c3.sh <libdir A> <libdir B> [<libdir C> ...]   (A against each of the rest)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
A=$1; shift
for B in "$@"; do
  timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-40} > gpurun_out/ab_c3_$B.txt 2>&1
  rc=$?; echo "ab $A vs $B rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_c3_$B.txt; [ $rc -eq 0 ] || exit $rc
done

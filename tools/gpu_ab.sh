# Same-box A/B of two library builds (tools/inproc_ab.py) on C3, C4 and the C3 dense container;
# then B becomes the in-tree library on the box (a scratch copy) and the GPU test suite and the
# default bench line run on it (tools/gpu_step.sh).
# usage: bash tools/gpu_ab.sh <libdir A> <libdir B>      (libdirs under shuffle-coding_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env..., iters
    local tag=$1; shift
    env "$@" timeout -k 10 300 python -u tools/inproc_ab.py $A $B ${ITERS:-40} > gpurun_out/ab_$tag.txt 2>&1
    local rc=$?; echo "ab $tag rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_$tag.txt; return $rc
}
A=$1; B=$2
run c3 AB_CONFIG=c3 || exit $?
ITERS=20 run c4 AB_CONFIG=c4 || exit $?
run dense AB_CONFIG=c3 AB_DENSE=1 || exit $?
if [ "$B" != lib ]; then cp shuffle-coding_amd/$B/libshufflecoding_amd.so shuffle-coding_amd/lib/; fi
bash tools/gpu_step.sh || exit $?

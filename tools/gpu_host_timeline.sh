# Kernel + memory-copy timeline of the host-memory leg (tools/host_trace.py) for one library
# build (installed as the in-tree library on the box), for tools/host_timeline.py.
# usage: bash tools/gpu_host_timeline.sh <libdir>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cp shuffle-coding_amd/$1/libshufflecoding_amd.so shuffle-coding_amd/lib/libshufflecoding_amd.so
timeout -s KILL 300 rocprofv3 --memory-copy-trace --kernel-trace -d gpurun_out/tl_$1 -o run --output-format csv -- python3 tools/host_trace.py 30 2 > gpurun_out/tl_$1.log 2>&1
rc=$?; echo "timeline rc=$rc"; grep "rep " gpurun_out/tl_$1.log; exit $rc

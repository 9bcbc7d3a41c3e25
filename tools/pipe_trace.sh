# Timeline of the host-buffer pipeline (kernels + memory copies) on C3, for tools/pipe_timeline.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe_trace
rm -rf gpurun_out/pipe_trace/t
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/pipe_trace/t -o run --output-format csv -- ./tools/pcie_bench 28 2 ${1:-64} > gpurun_out/pipe_trace/run.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/pipe_trace/run.log; exit $rc

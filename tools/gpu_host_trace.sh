# rocprofv3 runtime trace of the host-memory leg (tools/host_trace.py: HIP API calls, copies,
# kernels; no --pmc) and a kernel trace of the device-API variable-chunk test (which kernels it
# takes), each under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --stats -d gpurun_out/host_trace -o run --output-format csv -- python3 tools/host_trace.py 30 3 > gpurun_out/host_trace.log 2>&1
rc=$?; echo "host trace rc=$rc"; grep "rep " gpurun_out/host_trace.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/var_trace -o run --output-format csv -- python3 -m pytest -q -m gpu -p no:cacheprovider tests/test_gpu_parity.py -k "var_chunks_device_api" > gpurun_out/var_trace.log 2>&1
rc=$?; echo "var trace rc=$rc"; tail -2 gpurun_out/var_trace.log; exit $rc

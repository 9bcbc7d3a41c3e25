# Host-buffer pipeline: the whole GPU parity suite, then the PCIe-inclusive rate
# (C ABI caller, tools/pcie_bench.cpp, and Python caller, tools/pcie_rate.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pipe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pipe/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/pcie_bench 30 3 > gpurun_out/pipe/pcie_bench.log 2>&1
rc=$?; echo "pcie_bench rc=$rc"; tail -1 gpurun_out/pipe/pcie_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/pcie_rate.py 30 3 > gpurun_out/pipe/pcie_rate.log 2>&1
rc=$?; echo "pcie_rate rc=$rc"; tail -1 gpurun_out/pipe/pcie_rate.log; exit $rc

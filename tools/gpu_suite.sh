# Full GPU test suite, then the default bench line.  usage: bash tools/gpu_suite.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-suite}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json

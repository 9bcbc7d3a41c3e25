# GPU tests (optionally a -k / file selection), then the norm-range bench lines.
# usage: bash tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-t}; shift
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/${TAG}_tests.log
exit $rc

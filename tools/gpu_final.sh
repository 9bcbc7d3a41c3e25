set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
bash tools/final_round.sh r02k || exit 1

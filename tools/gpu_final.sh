set -o pipefail
cd $GRAFT_REPO_ROOT

bash tools/final_round.sh r02l || exit 1

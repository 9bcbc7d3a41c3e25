set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
AB_ITERS=40 bash tools/ab_round.sh "c3:lib_prev:lib c3:lib:lib_prev" || exit 1

# Round end: the whole GPU suite and smoke(), then the judged measurements (tools/final_round.sh)
# and the codecs bench with its kernel stats (tools/gpu_codecs_prof.sh, no PMC), all on the
# current build.   usage: bash tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-final}
bash tools/gpu_full.sh $TAG || exit 1
bash tools/final_round.sh $TAG || exit 1
NOPMC=1 bash tools/gpu_codecs_prof.sh $TAG || exit 1

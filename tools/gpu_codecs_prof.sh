# The section-4b fast kernels (ans_mfast.hpp) the way the headline is measured: tools/codecs_bench.py
# with Independent at 2^LI u8 symbols and Uniform / LogUniform at 2^LU u64 symbols, then its
# rocprofv3 kernel stats and the PMC passes (tools/pmc.sh) of the same command.
# usage: bash tools/gpu_codecs_prof.sh <tag> [LI=30] [LU=28]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-codecs}; LI=${2:-30}; LU=${3:-28}
OUT=gpurun_out/codecs_${TAG}
mkdir -p $OUT
timeout -k 10 300 python3 tools/codecs_bench.py $LI $LU > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 tools/codecs_bench.py $LI $LU > $OUT/stats.log 2>&1 || exit 1
echo stats done
if [ -z "$NOPMC" ]; then
  bash tools/pmc.sh codecs_${TAG} python3 tools/codecs_bench.py $LI $LU || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_codecs_${TAG} --config codecs --log2n $LI --json $OUT/pmc.json > $OUT/pmc_summary.txt
fi
echo done

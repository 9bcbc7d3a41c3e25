# One GPU call's worth of measurement: kernel stats + PMC passes (tools/pmc.sh) for the
# calibration kernel and the C3 / C4 benches.  usage: bash tools/prof_round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
for gap in 0 4; do
  bash tools/pmc.sh ${TAG}_calib$gap ./tools/hbm_calib $gap || exit 1
done
bash tools/pmc.sh ${TAG}_c3 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit 1
bash tools/pmc.sh ${TAG}_c4 python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_${TAG}_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/stats_${TAG}_c3.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_${TAG}_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/stats_${TAG}_c4.log 2>&1 || exit 1
for k in calib0 calib4; do python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_$k > gpurun_out/pmc_${TAG}_$k/summary.txt; done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_c3 --config c3 --log2n 30 --json gpurun_out/pmc_${TAG}_c3/pmc.json > gpurun_out/pmc_${TAG}_c3/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_c4 --config c4 --log2n 29 --json gpurun_out/pmc_${TAG}_c4/pmc.json > gpurun_out/pmc_${TAG}_c4/summary.txt
echo done

# The round's judged measurements in one GPU call: the driver-shaped bench line (C3 with the
# dense, C4 and host sub-objects and the CPU baseline), the rocprofv3 kernel stats of the C3 and
# C4 commands, and the PMC passes (tools/pmc.sh) whose per-launch HBM bytes and VALU counts
# bench.py reads from profiles/.
# usage: bash tools/final_round.sh <tag>      (then copy gpurun_out/final_<tag>/ into profiles/)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
export TMPDIR=/tmp
OUT=gpurun_out/final_${TAG}
mkdir -p $OUT
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
echo bench done
# the driver's shape (--steps 20 --warmup 5): the kernel stats of the headline's timed dispatches
# (kernel trace window: the dense pass's max(5, 20) + min(20, 10) dispatches and the 5 warm-up
# steps come first) -> profiles/*kstats*.json, which bench.py's frac_rocprof reads
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --no-host > $OUT/stats_c3.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c4 -o run --output-format csv -- python3 bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --no-host --no-dense > $OUT/stats_c4.log 2>&1 || exit 1
python3 tools/kstats_json.py $OUT/stats_c3/run_kernel_stats.csv $OUT/kstats_c3.json --config c3 --log2n 30 --trace $OUT/stats_c3/run_kernel_trace.csv --skip 35 --count 20 || exit 1
python3 tools/kstats_json.py $OUT/stats_c4/run_kernel_stats.csv $OUT/kstats_c4.json --config c4 --log2n 29 --trace $OUT/stats_c4/run_kernel_trace.csv --skip 5 --count 20 || exit 1
echo stats done
bash tools/pmc.sh ${TAG}_c3 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense --no-c4 --no-host || exit 1
bash tools/pmc.sh ${TAG}_c4 python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dense --no-c4 --no-host || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_c3 --config c3 --log2n 30 --json $OUT/pmc_c3.json > $OUT/pmc_c3_summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_c4 --config c4 --log2n 29 --json $OUT/pmc_c4.json > $OUT/pmc_c4_summary.txt
echo done

# Large-alphabet tables outside [2^16, 2^31] (r06): bench lines and kernel stats of C4's shape
# (2^29 u16 symbols, chunk 4096) under c4 (norm 134,561,356), c4s (4,096 symbols, norm 65,521)
# and c4b (65,536 symbols, norm 2^32 - 5), one box.   usage: bash tools/gpu_wide_norms.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-wide}
export TMPDIR=/tmp
OUT=gpurun_out/wide_${TAG}
mkdir -p $OUT
for cfg in c4 c4s c4b; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 5 --no-c4 --no-host --no-dense --no-cpu-baseline > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { tail -5 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['encode_ms'], d['decode_ms'], d['roofline']['kernel'])"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 20 --warmup 5 --no-c4 --no-host --no-dense --no-cpu-baseline > $OUT/stats_$cfg.log 2>&1 || exit 1
  python3 tools/kstats_json.py $OUT/stats_$cfg/run_kernel_stats.csv $OUT/kstats_$cfg.json --config $cfg --log2n 29 --trace $OUT/stats_$cfg/run_kernel_trace.csv --skip 5 --count 20 || exit 1
done
echo done

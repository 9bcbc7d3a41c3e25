# The C3 workload at norms outside [2^16, 2^31] (bench.py --config c3s / c3b): bench lines and
# rocprofv3 kernel stats.  usage: bash tools/gpu_norms.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-norms}
OUT=gpurun_out/norms_${TAG}
mkdir -p $OUT
for cfg in c3s c3b c3; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-c4 --no-host --no-dense \
      > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { tail -5 $OUT/bench_$cfg.err; exit 1; }
  echo "$cfg: $(python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print(d['value'],d['encode_ms'],d['decode_ms'],d['compressed_bytes_per_symbol'])")"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-c4 --no-host --no-dense > $OUT/stats_$cfg.log 2>&1 || exit 1
done
echo done

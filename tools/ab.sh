# A/B: run the GPU parity subset and the bench under each value of an env knob.
# usage: bash tools/ab.sh VAR "v1 v2 ..." [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; K=${3:-"crowded or random_tables or fast_kernel or golden or multiset or c3"}
mkdir -p gpurun_out
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/ab_${VAR}_${v}_tests.log 2>&1
  rc=$?; echo "$VAR=$v tests rc=$rc: $(tail -1 gpurun_out/ab_${VAR}_${v}_tests.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${VAR}_${v}_bench.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/ab_${VAR}_${v}_bench.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${VAR}_${v}_bench.log').read().strip().splitlines()[-1]); print('$VAR=$v', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])"
done

# C4 bench under each value of an env knob: bash tools/c4ab.sh VAR "v1 v2 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in $2; do
  export $1=$v
  timeout -k 10 300 python bench.py --config c4 --log2n 29 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c4ab_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/c4ab_$v.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4ab_$v.log').read().strip().splitlines()[-1]); print('$1=$v', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])"
done

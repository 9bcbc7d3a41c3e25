# bench at several sizes (occupancy sweep): bash tools/sizes.sh "28 29 30" [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in $1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --log2n $n ${@:2} > gpurun_out/size_$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/size_$n.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/size_$n.log').read().strip().splitlines()[-1]); print('log2n $n', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])"
done

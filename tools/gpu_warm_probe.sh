# The driver's bench command (--steps 20 --warmup 5) a few times beside --warmup 30, to see how
# much of the GPU's clock ramp the timed steps carry.  usage: bash tools/gpu_warm_probe.sh [extra bench flags]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 5 5 30 5; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup $w --no-cpu-baseline --no-host "$@" > gpurun_out/w.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/w.json').read().strip().splitlines()[-1]); print('warmup $w', d['value'], d['encode_ms'], d['decode_ms'], (d.get('dense') or {}).get('gib_s'), (d.get('c4') or {}).get('value'))"
done

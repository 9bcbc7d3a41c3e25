# Host-memory leg of two library builds, one after the other on one box (bench.py's host
# sub-object with each build as the in-tree library), then the GPU suite on B.
# usage: bash tools/gpu_host_ab.sh <libdir A> <libdir B>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=shuffle-coding_amd/lib/libshufflecoding_amd.so
for d in $1 $2 $1 $2; do
  cp shuffle-coding_amd/$d/libshufflecoding_amd.so $L
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-dense --no-c4 > gpurun_out/host_$d.json 2> gpurun_out/host_$d.err || { tail -5 gpurun_out/host_$d.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/host_$d.json').read().strip().splitlines()[-1])['host']; print('$d', d['gib_s'], d['encode_ms'], d['decode_ms'])"
done
bash tools/gpu_step.sh || exit $?

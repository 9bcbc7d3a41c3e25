# bench the C3 decode under alternative builds of the library: bash tools/libab.sh dir1 dir2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in "$@"; do
  if [ "$d" = default ]; then unset SHUFFLE_CODING_AMD_LIB; else export SHUFFLE_CODING_AMD_LIB=$PWD/shuffle-coding_amd/$d/libshufflecoding_amd.so; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/libab_$d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/libab_$d.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/libab_$d.log').read().strip().splitlines()[-1]); print('$d', 'value', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])"
done

# C3 over chunk lengths (sweep 1024-16384): one bench line each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/chunk_sweep.jsonl
for L in 1024 2048 4096 8192 16384; do
  timeout -k 10 200 python3 bench.py --chunk-len $L --steps 15 --warmup 8 --no-cpu-baseline --no-dense > gpurun_out/sweep_$L.log 2>&1 || { tail -3 gpurun_out/sweep_$L.log; exit 1; }
  grep '^{' gpurun_out/sweep_$L.log >> gpurun_out/chunk_sweep.jsonl
done
echo done

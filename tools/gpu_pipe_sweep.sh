# Host-memory pipeline sweep (tools/host_trace.py: C3 from and to page-locked host memory, 3
# round trips per process) over pipeline depth and batch size, one build installed as the
# in-tree library.  usage: bash tools/gpu_pipe_sweep.sh <libdir> "<depth:MiB> ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cp shuffle-coding_amd/$1/libshufflecoding_amd.so shuffle-coding_amd/lib/libshufflecoding_amd.so
for cfg in $2; do
  IFS=: read d mb <<< "$cfg"
  ANS_PIPE_DEPTH=$d HT_BATCH_MB=$mb timeout -k 10 120 python3 tools/host_trace.py 30 3 > gpurun_out/sweep_$cfg.log 2>&1 || { echo "$cfg failed"; tail -3 gpurun_out/sweep_$cfg.log; exit 1; }
  echo "$cfg $(grep 'rep ' gpurun_out/sweep_$cfg.log | tail -2 | tr '\n' ' ')"
done

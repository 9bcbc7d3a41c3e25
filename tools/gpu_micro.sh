set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench > gpurun_out/microbench.txt 2>&1; echo "micro rc=$?"; cat gpurun_out/microbench.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_v1.log 2>&1; echo "prof rc=$?"
tail -3 gpurun_out/prof_v1.log
find gpurun_out/prof_v1 -name "*stats*" | head

# Rehearses bench.py's N>1 path on a 1-GPU box: 2 ranks share device 0, gloo for the barrier
# and the max over ranks (the driver's real run uses one GPU per rank and RCCL).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BENCH_SHARE_DEVICE=1 BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --log2n 28 > gpurun_out/mgpu.log 2>&1
rc=$?; echo "mgpu rc=$rc"; tail -2 gpurun_out/mgpu.log; exit $rc

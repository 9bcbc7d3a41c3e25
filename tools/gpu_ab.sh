# Same-box A/B of two library builds (tools/inproc_ab.py) on C3 and C4, then the GPU test
# suite, the default bench line and one PMC pass (instruction counts) of the C3 kernels.
# usage: bash tools/gpu_ab.sh <libdir A> <libdir B>      (libdirs under shuffle-coding_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/inproc_ab.py $1 $2 40 > gpurun_out/ab_c3.txt 2>&1
rc=$?; echo "ab c3 rc=$rc"; cat gpurun_out/ab_c3.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=c4 timeout -k 10 300 python -u tools/inproc_ab.py $1 $2 20 > gpurun_out/ab_c4.txt 2>&1
rc=$?; echo "ab c4 rc=$rc"; cat gpurun_out/ab_c4.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_step.sh || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_ab -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 --no-host --no-dense > gpurun_out/pmc_ab.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc

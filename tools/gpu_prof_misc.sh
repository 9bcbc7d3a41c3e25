# Kernel times of the section-4b codecs (tools/codecs_bench.py) and two PMC passes over the
# C3 slot and dense round trips (instruction counts; DRAM-side bytes), each under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_codecs -o run --output-format csv -- python3 tools/codecs_bench.py 26 24 > gpurun_out/prof_codecs.log 2>&1
rc=$?; echo "codecs prof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_codecs.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_dense1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 --no-host > gpurun_out/pmc_dense1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B -d gpurun_out/pmc_dense2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 --no-host > gpurun_out/pmc_dense2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; exit $rc

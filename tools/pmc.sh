# rocprofv3 PMC passes over one command (one counter group per pass, --kernel-trace only;
# never combined with sys/runtime traces).  The memory-side byte counts come from the TCC's
# request-size counters (MI355X_MICROARCH.md §HBM; tools/pmc_summary.py explains the sums).
# usage: bash tools/pmc.sh <tag> <command...>     (e.g. python3 bench.py --steps 2 --warmup 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_${TAG}
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
  "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" \
  "TCC_HIT TCC_MISS TCC_REQ TCC_READ_REQ" ; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_${TAG}/p$i -o run --output-format csv -- "$@" > gpurun_out/pmc_${TAG}/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_${TAG}/p$i.log; exit $rc; }
done

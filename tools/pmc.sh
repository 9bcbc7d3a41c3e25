# rocprofv3 PMC passes (one counter group per pass, --kernel-trace only; never with sys/runtime traces)
# usage: bash tools/pmc.sh <tag> [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}; shift
# PMC_META: e.g. "--config c3 --log2n 30" (recorded in pmc.json for bench.py)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_${TAG}
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_${TAG}/p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_${TAG}/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_${TAG}/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG} --json gpurun_out/pmc_${TAG}/pmc.json ${PMC_META} | tee gpurun_out/pmc_${TAG}/summary.txt

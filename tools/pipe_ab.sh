# A/B of the page-locked copy engine (kernels vs runtime copies) in one box session
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pipeline or dense_and_slot or golden" > gpurun_out/pipe/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/pipe/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 256; do
for m in kernel runtime kernel runtime; do
ANS_PIPE_COPY=$m timeout -k 10 120 ./tools/pcie_bench 30 3 $b > gpurun_out/pipe/ab_${m}_$b.log 2>&1
rc=$?; echo "$m $b rc=$rc $(tail -1 gpurun_out/pipe/ab_${m}_$b.log | cut -c90-)"; [ $rc -eq 0 ] || exit $rc
done; done

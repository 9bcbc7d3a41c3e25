# Full GPU check: parity suite, smoke, bench (with CPU baseline), kernel-trace profile, PMC,
# PCIe-inclusive rate, C4 bench.  usage: bash tools/full_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
PMC_META="--config c3 --log2n 30" bash tools/pmc.sh $TAG > $O/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail $O/pmc.log; exit $rc; }
timeout -k 10 600 python tools/pcie_rate.py 30 3 > $O/pcie.log 2>&1
rc=$?; echo "pcie rc=$rc"; tail -1 $O/pcie.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --log2n 29 --steps 5 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 $O/c4.log

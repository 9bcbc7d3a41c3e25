# One PMC pass of wave-state counters (issue vs waiting) over a bench config with the in-tree
# library.  usage: bash tools/pmc_wait.sh <tag> <config>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw_$1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/pmcw_$1 -o run --output-format csv -- python3 bench.py --config $2 --steps 2 --warmup 1 --no-cpu-baseline --no-dense --no-c4 --no-host > gpurun_out/pmcw_$1/log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcw_$1/log; exit $rc; }
python3 - $1 <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/pmcw_{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("<")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if d.get("SQ_WAVES", 0) < 1000: continue
    w = d["SQ_WAVE_CYCLES"]
    print(k, {c: round(v / d["SQ_WAVES"]) for c, v in d.items()}, "wait_any %.2f wait_inst %.2f active %.2f" % (d["SQ_WAIT_ANY"] / w, d["SQ_WAIT_INST_ANY"] / w, d["SQ_ACTIVE_INST_ANY"] / w))
PY

# FETCH_SIZE / WRITE_SIZE calibration for the fast kernels' access pattern (tools/hbm_calib.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for gap in 0 4; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/calib/${ctr}_$gap -o run --output-format csv -- ./tools/hbm_calib $gap > gpurun_out/calib/${ctr}_$gap.log 2>&1
    rc=$?; echo "$ctr gap $gap rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/calib/${ctr}_$gap.log; exit $rc; }
    grep "gap" gpurun_out/calib/${ctr}_$gap.log | tail -1
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/calib/*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        per[(row["Kernel_Name"][:6], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in sorted(per.items()):
        print(f, k, d, c, "%.4g KiB = %.4f x 2^30 B" % (v, v * 1024 / 2**30))
PY

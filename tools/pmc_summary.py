#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes per kernel (mean over dispatches).

HBM bytes follow MI355X_MICROARCH.md §HBM.  FETCH_SIZE (KiB) counts memory-side read
requests at 64 B.  For wide coalesced streaming reads on gfx950 it reports half of the bytes
(the guide's x2 rule).  For other patterns the guide says to calibrate on a known byte count.
tools/hbm_calib.hip does that for the fast kernels' pattern (64 B per lane, lanes one chunk
apart, thousands of cycles between a lane's groups) and measures x1.00 (profiles/r01_hbm_calib.txt).
So --fetch-factor selects the factor: `traffic` uses the calibrated factor, and the x2 figure
is reported beside it as an upper bound.  WRITE_SIZE is exact (calibrated x1.00).
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict


def short(name):
    for key in ("k_encode", "k_decode", "k_gen_iid", "k_compact"):
        if key in name:
            return ("fast::" if "fast::" in name else "") + key
    return name[:40]


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
    out = {}
    for k, cs in sorted(vals.items()):
        if "k_encode" not in k and "k_decode" not in k:
            continue
        agg = {}
        for c, lst in cs.items():
            per = defaultdict(float)
            for d, v in lst:
                per[d] += v  # sum over XCD / instances within one dispatch
            agg[c] = sum(per.values()) / len(per)
        out[k] = agg
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json", help="write per-kernel HBM bytes per launch here (bench.py roofline.traffic)")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--log2n", type=int, default=None)
    ap.add_argument("--chunk-len", type=int, default=4096)
    ap.add_argument("--fetch-factor", type=float, default=1.0,
                    help="bytes per FETCH_SIZE byte for this access pattern (tools/hbm_calib.hip)")
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(__file__), "..", "shuffle-coding_amd", "lib",
                                                  "libshufflecoding_amd.so"))
    a = ap.parse_args()
    out = summarise(a.root)
    kernels = {}
    for k, agg in out.items():
        print(f"== {k}")
        for c in sorted(agg):
            print(f"   {c:24s} {agg[c]:.4g}")
        raw_rd = agg["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in agg else None
        rd = a.fetch_factor * raw_rd if raw_rd is not None else None
        wr = agg["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in agg else None
        if rd is not None:
            print(f"   HBM read  ({a.fetch_factor:g}*FETCH_SIZE) {rd / 1e9:.4f} GB   (x2 rule: {2 * raw_rd / 1e9:.4f} GB)")
        if wr is not None:
            print(f"   HBM write (WRITE_SIZE)   {wr / 1e9:.4f} GB")
        if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
            print(f"   VALU instr per wave      {agg['SQ_INSTS_VALU'] / agg['SQ_WAVES']:.0f}")
        if rd is not None and wr is not None:
            key = k.replace("fast::", "")
            kernels[key] = {"hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                            "hbm_bytes_per_launch_x2_rule": 2 * raw_rd + wr, "fetch_factor": a.fetch_factor,
                            "counters": agg}
    if a.json:
        with open(a.lib, "rb") as f:
            lib_hash = hashlib.sha256(f.read()).hexdigest()[:16]
        with open(a.json, "w") as f:
            json.dump({"config": a.config, "log2n": a.log2n, "chunk_len": a.chunk_len, "lib_hash": lib_hash,
                       "method": "rocprofv3 --kernel-trace --pmc, one counter group per pass; HBM bytes = "
                                 "fetch_factor*FETCH_SIZE + WRITE_SIZE (KiB x 1024); fetch_factor calibrated "
                                 "by tools/hbm_calib.hip (MI355X_MICROARCH.md: calibrate other patterns)",
                       "kernels": kernels}, f, indent=1)


if __name__ == "__main__":
    main()

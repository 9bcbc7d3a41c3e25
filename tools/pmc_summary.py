#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes (tools/pmc.sh) per kernel, mean over dispatches.

Memory-side bytes come from the TCC's request counters, summed over the 16 channels x 8 XCDs
of a dispatch (MI355X_MICROARCH.md §HBM):
  * reads, by request size: 32*TCC_EA0_RDREQ_32B + 64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B.
    FETCH_SIZE's own expression tallies 128-B requests through TCC_BUBBLE, which gfx950 does
    not count for streaming reads: that is the guide's "FETCH_SIZE reports half" rule.
  * reads that went to DRAM: 32*TCC_EA0_RDREQ_DRAM_32B (the counter counts 32-B units).
  * writes: 32*(TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B) + 64*TCC_EA0_WRREQ_64B (WRITE_SIZE's
    expression) and, DRAM-side, 32*TCC_EA0_WRREQ_WRITE_DRAM_32B.
tools/hbm_calib.hip moves exactly 2^30 bytes in the fast kernels' access pattern; its rows in
the summary show which sums read true (profiles/r02_hbm_calib.txt).
"""
import argparse
import csv
import glob
import hashlib
import json
import os
from collections import defaultdict

KEYS = ("k_encode_w", "k_encode", "k_decode_g", "k_decode_w", "k_decode", "k_gen_iid", "k_compact", "k_sample_iid")


def short(name):
    base = name.split("(")[0]
    for key in ("k_menc", "k_mdec"):  # ans_mfast.hpp: one kernel per codec model
        if key in base:
            for model in ("IndepModel", "LogUniformModel", "UniformModel"):
                if model in base:
                    return f"mfast::{key}<{model}>"
    for key in KEYS:
        if key in base:
            return ("fast::" if "fast::" in base else "") + key
    if base.strip().endswith(" rd") or base.strip() == "rd":
        return "calib_rd"
    if base.strip().endswith(" wr") or base.strip() == "wr":
        return "calib_wr"
    return base[-40:]


def durations(root):
    """Mean kernel duration (ns) per short name from the kernel traces of every pass."""
    d = defaultdict(list)
    for f in glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                d[short(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
    out = {}
    for k, cs in sorted(vals.items()):
        agg = {}
        for c, lst in cs.items():
            per = defaultdict(float)
            for d, v in lst:
                per[d] += v  # sum over channels / XCDs within one dispatch
            agg[c] = sum(per.values()) / len(per)
        out[k] = agg
    return out


def derive(agg, dur_ns):
    g = agg.get
    r = {}
    if all(x in agg for x in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B")):
        r["read_bytes_by_size"] = 32 * g("TCC_EA0_RDREQ_32B") + 64 * g("TCC_EA0_RDREQ_64B") + 128 * g("TCC_EA0_RDREQ_128B")
        if "TCC_EA0_RDREQ" in agg:
            r["read_requests_unsized"] = g("TCC_EA0_RDREQ") - g("TCC_EA0_RDREQ_32B") - g("TCC_EA0_RDREQ_64B") - g("TCC_EA0_RDREQ_128B")
    if "TCC_EA0_RDREQ_DRAM_32B" in agg:
        r["read_bytes_dram"] = 32 * g("TCC_EA0_RDREQ_DRAM_32B")
    if "TCC_EA0_WRREQ" in agg and "TCC_EA0_WRREQ_64B" in agg:
        r["write_bytes"] = 32 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B")) + 64 * g("TCC_EA0_WRREQ_64B")
    if "TCC_EA0_WRREQ_WRITE_DRAM_32B" in agg:
        r["write_bytes_dram"] = 32 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B")
    if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
        r["valu_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
    if "TCC_HIT" in agg and "TCC_MISS" in agg and g("TCC_HIT") + g("TCC_MISS") > 0:
        r["l2_hit_rate"] = g("TCC_HIT") / (g("TCC_HIT") + g("TCC_MISS"))
    if dur_ns:
        r["duration_ns"] = dur_ns
        if "GRBM_GUI_ACTIVE" in agg:
            r["clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8 / dur_ns  # summed over the 8 XCDs
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json", help="write per-kernel bytes per launch here (bench.py roofline.traffic / .valu)")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--log2n", type=int, default=None)
    ap.add_argument("--chunk-len", type=int, default=4096)
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(__file__), "..", "shuffle-coding_amd", "lib",
                                                  "libshufflecoding_amd.so"))
    a = ap.parse_args()
    out = summarise(a.root)
    durs = durations(a.root)
    kernels = {}
    for k, agg in out.items():
        d = derive(agg, durs.get(k))
        print(f"== {k}")
        for c in sorted(agg):
            print(f"   {c:30s} {agg[c]:.4g}")
        for c in sorted(d):
            v = d[c]
            print(f"   -> {c:27s} {v / 1e9:.4f} GB" if "bytes" in c else f"   -> {c:27s} {v:.4g}")
        if "read_bytes_by_size" in d and "write_bytes" in d:
            rd = d.get("read_bytes_dram", d["read_bytes_by_size"])
            kernels[k.replace("fast::", "")] = {
                "hbm_read_bytes": rd, "hbm_write_bytes": d.get("write_bytes_dram", d["write_bytes"]),
                "hbm_bytes_per_launch": rd + d.get("write_bytes_dram", d["write_bytes"]),
                "derived": d, "counters": agg}
    if a.json:
        with open(a.lib, "rb") as f:
            lib_hash = hashlib.sha256(f.read()).hexdigest()[:16]
        with open(a.json, "w") as f:
            json.dump({"config": a.config, "log2n": a.log2n, "chunk_len": a.chunk_len, "lib_hash": lib_hash,
                       "method": "rocprofv3 --kernel-trace --pmc, one counter group per pass (tools/pmc.sh); "
                                 "HBM bytes = 32*TCC_EA0_RDREQ_DRAM_32B + 32*TCC_EA0_WRREQ_WRITE_DRAM_32B per "
                                 "dispatch, summed over channels and XCDs; request-size sums beside them; "
                                 "calibrated on tools/hbm_calib.hip (profiles/r02_hbm_calib.txt)",
                       "kernels": kernels}, f, indent=1)


if __name__ == "__main__":
    main()

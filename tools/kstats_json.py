#!/usr/bin/env python3
"""Kernel averages of a rocprofv3 --kernel-trace --stats run (its kernel_stats.csv) as the JSON
record bench.py reads for roofline.frac_rocprof (profiles/*kstats*.json): per short kernel name
(tools/pmc_summary.py's names) the calls, average, minimum and maximum duration over every
dispatch of the run, tagged with the workload and the sha256 prefix of the library that ran.
usage: python tools/kstats_json.py <kernel_stats.csv> <out.json> [--config c3 --log2n 30 --chunk-len 4096]
       [--trace <kernel_trace.csv> --skip S --count K]
With --trace, each kernel's record averages its dispatches S .. S+K-1 (in dispatch order) from the
per-dispatch trace of the same run: for bench.py --steps K --warmup W with the dense pass
(max(W, 20) + min(K, 10) dispatches of the coding kernels before the headline's), S = that + W
selects exactly the K dispatches the headline's HIP events time.
"""
import argparse
import csv
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("out")
    p.add_argument("--config", default="c3")
    p.add_argument("--log2n", type=int, default=30)
    p.add_argument("--chunk-len", type=int, default=4096)
    p.add_argument("--lib", default=os.path.join(ROOT, "shuffle-coding_amd", "lib", "libshufflecoding_amd.so"))
    p.add_argument("--trace", default=None, help="rocprofv3 kernel_trace.csv of the same run")
    p.add_argument("--skip", type=int, default=0)
    p.add_argument("--count", type=int, default=0)
    a = p.parse_args()
    kernels = {}
    with open(a.csv) as fh:
        for row in csv.DictReader(fh):
            k = short(row["Name"]).replace("fast::", "")  # bench.py kernel_name()
            calls = int(row["Calls"])
            prev = kernels.get(k)
            if prev is not None:  # several instantiations under one short name: the busiest one
                if prev["calls"] * prev["avg_ns"] >= calls * float(row["AverageNs"]):
                    continue
            kernels[k] = {"calls": calls, "avg_ns": float(row["AverageNs"]), "min_ns": float(row["MinNs"]),
                          "max_ns": float(row["MaxNs"]), "name": row["Name"][:160]}
    method = ("rocprofv3 --kernel-trace --stats of the bench command; averages over every dispatch "
              "(warm-up and sub-object launches of the same kernel included)")
    if a.trace:
        per = {}
        with open(a.trace) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
        for row in rows:
            k = short(row["Kernel_Name"]).replace("fast::", "")
            per.setdefault(k, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for k, rec in kernels.items():
            d = per.get(k, [])[a.skip:a.skip + a.count] if a.count else per.get(k, [])[a.skip:]
            if not d:
                continue
            rec["all_dispatches"] = {x: rec[x] for x in ("calls", "avg_ns", "min_ns", "max_ns")}
            rec.update(calls=len(d), avg_ns=sum(d) / len(d), min_ns=float(min(d)), max_ns=float(max(d)),
                       dispatch_window=[a.skip, a.skip + len(d)])
        method = (f"rocprofv3 --kernel-trace --stats of the bench command; avg_ns over dispatches "
                  f"[{a.skip}, {a.skip + a.count}) of each kernel from the same run's kernel trace: the "
                  f"headline's timed steps (the --stats average over every dispatch is kept as all_dispatches)")
    with open(a.lib, "rb") as f:
        lib_hash = hashlib.sha256(f.read()).hexdigest()[:16]
    rec = {"config": a.config, "log2n": a.log2n, "chunk_len": a.chunk_len, "lib_hash": lib_hash,
           "method": method, "src": os.path.relpath(os.path.abspath(a.csv), ROOT), "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: round(v["avg_ns"]) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Prints the kernel / memory-copy timeline of the last host-memory round trip in a rocprofv3
--kernel-trace --memory-copy-trace run of tools/host_trace.py (tools/gpu_host_timeline.sh):
one line per operation, times in ms from the round trip's first operation.
usage: python3 tools/host_timeline.py gpurun_out/tl_<libdir>
"""
import csv
import glob
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    ops = []
    for r in rows(os.path.join(d, "**", "*kernel_trace.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("shuffle_coding::", "")
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + name[:48], r.get("Stream_Id", "")))
    for r in rows(os.path.join(d, "**", "*memory_copy_trace.csv")):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r["Direction"], r.get("Stream_Id", "")))
    ops.sort()
    # the last round trip: from the last encode kernel group's first H2D copy
    enc = [i for i, o in enumerate(ops) if "k_encode" in o[2]]
    first_enc_of_last = enc[-1]
    while first_enc_of_last > 0 and any("k_encode" in ops[j][2] for j in range(max(0, first_enc_of_last - 6), first_enc_of_last)):
        first_enc_of_last -= 1
    i0 = first_enc_of_last
    while i0 > 0 and "HOST_TO_DEVICE" in ops[i0 - 1][2]:
        i0 -= 1
    t0 = ops[i0][0]
    for s, e, name, st in ops[i0:]:
        if (e - s) < 20000 and name.startswith("C"):  # small metadata copies
            continue
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  s{st:>3} {name}")


if __name__ == "__main__":
    main()

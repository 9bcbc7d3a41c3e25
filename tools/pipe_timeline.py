"""Prints the tail of a rocprofv3 kernel + memory-copy trace as a timeline (ms from the
first event of the window): which copies and kernels overlap in the host-buffer pipeline.
usage: python tools/pipe_timeline.py <trace dir> [last_n_events]"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    ev = []
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nb = r.get("Size") or ""
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       r["Direction"].replace("MEMORY_COPY_", ""), r["Stream_Id"], nb))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("<")[0].split("(")[0].replace("shuffle_coding::", "")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r["Stream_Id"], r["Grid_Size_X"]))
    ev.sort()
    ev = ev[-last:]
    t0 = ev[0][0]
    for s, e, what, stream, extra in ev:
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:7.3f}  s{stream:>2} {what:24s} {extra}")


if __name__ == "__main__":
    main()

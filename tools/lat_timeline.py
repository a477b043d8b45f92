"""Lay out the kernels and memory copies of a rocprofv3 trace (CSV) of
tools/lat_trace.py: the last N dispatches / copies, times relative to the
first of them (development tool)."""
import csv
import glob
import sys

root = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ev = []
for path in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:34], r.get("Stream_Id", "")))
for path in glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?"), ""))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, name, st in ev:
    print(f"{name:40s} {st:>4} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us")

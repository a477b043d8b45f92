"""Kernel timeline of a rocprofv3 --kernel-trace CSV (development tool):
per-kernel start/end relative to the first k_verify_q of the timed steps,
and the device-idle gaps between consecutive verify steps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[:28], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
         for r in rows]
qs = [i for i, (n, s, e) in enumerate(names) if n.startswith("k_verify_q")]
# optional 2nd argument: verify steps to drop from the end (bench.py runs 5
# synchronous calls for the roofline after its timed region)
if len(sys.argv) > 2:
    qs = qs[:len(qs) - int(sys.argv[2])]
if len(qs) < 3:
    sys.exit("too few steps")
t0 = names[qs[-3]][2]  # end of the third-last step
for n, s, e in names:
    if s >= t0 - 50_000 and s <= names[qs[-1]][2]:
        print(f"{n:28s} start {(s - t0) / 1e3:9.1f} us  end {(e - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}")

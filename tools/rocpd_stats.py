"""Kernel statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats` on ROCm 7.2 when no --output-format is
given), written in the layout of rocprofv3's own kernel_stats.csv:

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_bench_kernel_stats.csv

Durations are nanoseconds, as in rocprofv3's CSV.
"""
from __future__ import annotations

import csv
import sqlite3
import sys


def kernel_stats(db: str) -> list[dict]:
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [{"Name": n, "Calls": c, "TotalDurationNs": s, "AverageNs": round(a, 1),
             "Percentage": round(100.0 * s / total, 4), "MinNs": lo, "MaxNs": hi}
            for n, c, s, a, lo, hi in rows]


def main() -> None:
    rows = kernel_stats(sys.argv[1])
    w = csv.DictWriter(sys.stdout, fieldnames=list(rows[0]))
    w.writeheader()
    w.writerows(rows)


if __name__ == "__main__":
    main()

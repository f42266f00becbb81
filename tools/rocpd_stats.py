#!/usr/bin/env python3
"""Per-kernel statistics (calls, total/avg ms, share) from a rocprofv3 rocpd database (the default
output format of rocprofv3 --kernel-trace on ROCm 7), written as the kernel_stats.csv layout.
usage: rocpd_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys


def main() -> int:
    db = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                      f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, c, s, a, lo, hi in rows:
        w.writerow([n, c, s, round(a, 1), round(100.0 * s / total, 3), lo, hi])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""Export the per-kernel summary of a rocprofv3 rocpd database (``--kernel-trace --stats`` run
written as ``<dir>/<name>_results.db``) to a CSV like rocprofv3's ``kernel_stats.csv``.

usage: python tools/prof_summary.py gpurun_out/prof_r1d/run_results.db profiles/r01_d_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def summarize(db_path):
    con = sqlite3.connect(db_path)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    out = []
    for name, calls, tot, avg, mn, mx in rows:
        out.append({"Name": name, "Calls": calls, "TotalDurationNs": int(tot), "AverageNs": round(avg, 1),
                    "Percentage": round(100.0 * tot / total, 4), "MinNs": int(mn), "MaxNs": int(mx)})
    return out


def main():
    if len(sys.argv) != 3:
        sys.exit(__doc__)
    rows = summarize(sys.argv[1])
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:12]:
        print(f"{r['Percentage']:7.2f}%  {r['Calls']:6d}  {r['AverageNs'] / 1e3:9.2f} us  {r['Name'][:90]}")


if __name__ == "__main__":
    main()

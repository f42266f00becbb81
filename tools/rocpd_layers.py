#!/usr/bin/env python3
"""Per-position kernel timing of U-Net evaluations from a rocprofv3 rocpd database (kernel trace of a
one-lane sampling pass): a pass starts at k_first_acf.  Passes are grouped by their kernel count and
the grids of all their kernels, so an evaluation split into passes of different sizes (config 5's 2 GiB
cap: an 84-image and a 44-image pass per Bt = 128 evaluation) is reported pass by pass, never as one
median over both.  usage: rocpd_layers.py run_results.db [out.txt]"""
import collections
import sqlite3
import statistics
import sys


def short(n: str) -> str:
    n = n.replace("void ", "").replace("tcx::(anonymous namespace)::", "")
    return n.split("(tcx::")[0].split("(float")[0].split("(double")[0].split("(int")[0].split("(unsigned")[0][:60]


def main() -> int:
    db = sqlite3.connect(sys.argv[1])
    try:
        rows = db.execute("select name, start, end, grid_x * 1000003 + grid_y * 1009 + grid_z from kernels order by start").fetchall()
    except sqlite3.OperationalError:
        rows = db.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    rows = [r for r in rows if "tcx::" in r[0]]
    seq, cur = [], []
    for r in rows:
        if "k_first_acf" in r[0] and cur:
            seq.append(cur)
            cur = []
        cur.append(r)
    seq.append(cur)
    L = collections.Counter(len(s) for s in seq).most_common(1)[0][0]
    groups = collections.defaultdict(list)
    for s in seq:
        if len(s) == L:
            groups[tuple(r[3] for r in s)].append(s)  # the pass's grid signature (its row count)
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    total_span = 0.0
    for gk in sorted(groups, reverse=True):
        ev = groups[gk]
        ev = ev[min(5, len(ev) // 2):]  # skip warm-up passes
        tot = 0.0
        print(f"== pass kind {sorted(groups, reverse=True).index(gk)}: conv grid key {gk[4]} ({len(ev)} passes)", file=out)
        for i in range(L):
            d = statistics.median((s[i][2] - s[i][1]) / 1e3 for s in ev)
            tot += d
            print(f"{i:2d} {short(ev[0][i][0]):60s} grid={ev[0][i][3] // 1000003:>8d} {d:9.1f} us", file=out)
        span = statistics.median((s[-1][2] - s[0][1]) / 1e3 for s in ev)
        total_span += span
        print(f"sum of kernel medians {tot:.1f} us; first-start..last-end {span:.1f} us per pass ({len(ev)} passes)",
              file=out)
    if len(groups) > 1:
        print(f"per evaluation (one pass of each kind): {total_span:.1f} us", file=out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

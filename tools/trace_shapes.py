"""Per-(kernel, grid) duration table from a rocprofv3 --kernel-trace database (profiling helper)."""
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, workgroup_x, count(*), avg(duration), sum(duration) from kernels "
                 "group by name, grid_x, grid_y order by sum(duration) desc limit ?", (n,)).fetchall()
for r in rows:
    name = r[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("tcx::", "")
    print(f"{name[-44:]:>44} grid=({r[1]},{r[2]}) wg={r[3]} n={r[4]:5d} avg={r[5] / 1000:7.2f} us "
          f"sum={r[6] / 1e6:7.2f} ms")

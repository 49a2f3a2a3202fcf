"""Summarise a rocprofv3 kernel-trace database: per-kernel totals (and per grid size with --grid)."""
import sqlite3
import sys

db = sys.argv[1]
by_grid = "--grid" in sys.argv
con = sqlite3.connect(db)
cur = con.cursor()
key = "name, grid_x" if by_grid else "name"
rows = cur.execute(f"select {key}, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels group by {key} "
                   f"order by sum(duration) desc").fetchall()
tot = sum(r[-2] for r in rows)
print(f"total kernel time {tot:.2f} ms over {sum(r[-3] for r in rows)} dispatches")
print(f"{'ms':>9} {'%':>5} {'calls':>6} {'avg_us':>9}  kernel")
for r in rows[: int(dict(a.split('=') for a in sys.argv[2:] if a.startswith('top=')).get('top', 30))]:
    name = r[0][:90]
    g = f" grid={r[1]}" if by_grid else ""
    print(f"{r[-2]:9.2f} {100 * r[-2] / tot:5.1f} {r[-3]:6d} {r[-1]:9.1f}  {name}{g}")

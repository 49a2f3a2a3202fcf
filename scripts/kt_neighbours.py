"""For every launch of kernels whose name contains a pattern, count the kernels launched just
before and after it (rocprofv3 kernel-trace CSV, in dispatch order): which op issues a copy."""
import collections
import csv
import sys

path, pat = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(path)))
key = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Timestamp"
rows.sort(key=lambda r: int(r[key]))
names = [r["Kernel_Name"] for r in rows]
grids = [r.get("Grid_Size_X", r.get("Grid_Size", "")) for r in rows]
c = collections.Counter()
for i, nm in enumerate(names):
    if pat in nm:
        prev = names[i - 1][:90] if i else "-"
        nxt = names[i + 1][:90] if i + 1 < len(names) else "-"
        c[(grids[i], prev, nxt)] += 1
for (g, p, n), k in c.most_common(25):
    print(f"{k:6d} grid={g:>8}  before: {p}\n{'':22}after:  {n}")

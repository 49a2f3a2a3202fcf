"""Print a rocprofv3 *_kernel_stats.csv: average us, calls, name (optional substring filter)."""
import csv
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in csv.DictReader(open(sys.argv[1])):
    if flt in r["Name"]:
        print(f"{float(r['AverageNs']) / 1e3:9.1f} us x{r['Calls']:>5}  {r['Name'][:100]}")

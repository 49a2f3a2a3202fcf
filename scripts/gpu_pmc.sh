#!/bin/bash
# PMC passes (one counter group per run) over a short program: PMC_GROUPS="A,B C,D" PROG="python3 x.py"
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for grp in $PMC_GROUPS; do
  i=$((i+1))
  ctrs=$(echo $grp | tr ',' ' ')
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d /tmp/pmc$i -o p -- $PROG > gpurun_out/pmc/run$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/run$i.log; exit 1; }
  f=$(find /tmp/pmc$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$PMC_FILTER" <<'PY'
import csv, sys, collections
f, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if filt in r['Kernel_Name']:
        agg[(r['Kernel_Name'][:60], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    v.sort()
    print(f"{c:28s} median {v[len(v)//2]:16.1f}  n={len(v)}  {k}")
PY
done

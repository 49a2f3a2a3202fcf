#!/bin/bash
# rocprofv3 kernel-trace of a short bench + PMC passes (one counter group per run) on the dominant kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P=/tmp/prof; mkdir -p $P gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bench -o bench -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_stdout.log 2> gpurun_out/prof/bench_stderr.log || { echo "bench prof rc $?"; tail -20 gpurun_out/prof/bench_stderr.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/roof -o roof -- python3 -u scripts/roof_kernel.py 20 > gpurun_out/prof/roof.log 2>&1 || { echo "roof rc $?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o fetch -- python3 -u scripts/roof_kernel.py 5 > gpurun_out/prof/pmc_fetch.log 2>&1 || { echo "fetch rc $?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_write -o write -- python3 -u scripts/roof_kernel.py 5 > gpurun_out/prof/pmc_write.log 2>&1 || { echo "write rc $?"; exit 1; }
find $P -type f -exec ls -la {} \;
for f in $(find $P -name "*stats.csv" -o -name "*counter_collection.csv"); do cp $f gpurun_out/prof/; done
# per-kernel-grid summary of the bench trace
python3 - <<'PY' > gpurun_out/prof/bench_by_kernel.txt
import csv, glob, collections
f = glob.glob('/tmp/prof/bench/**/*kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    k = (r['Kernel_Name'][:100], r.get('Grid_Size_X', r.get('Grid_Size', '')))
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[k][0] += 1; agg[k][1] += d
tot = sum(v[1] for v in agg.values())
print(f"total {tot/1e3:.1f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:80]:
    print(f"{v[1]/1e3:9.2f} ms {100*v[1]/tot:5.1f}% {v[0]:6d} {v[1]/v[0]:9.1f}us grid={k[1]} {k[0]}")
PY
ls -la gpurun_out/prof

#!/bin/bash
# Bench line (BENCH_ARGS; NOBENCH=1 skips it), then per config in TRACES (default "c3 c2") a rocprofv3
# kernel trace of one generation after a warm-up (c3: B = 8, c2: B = 1, c5: B = 4 at 768^2),
# summarised per family and per kernel + grid (scripts/kt_summary.py) into
# gpurun_out/prof/<cfg>_by_kernel.txt, with the gzipped trace and the --stats CSV beside it.
# LEDGER=1 adds the per-shape step ledgers of c3 / c2 (scripts/ledger.py) to gpurun_out/prof/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
if [ -z "$NOBENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -4 gpurun_out/bench.err; cat gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${TRACES-c3 c2}; do
  case $cfg in
    c3) A="--batch 8" ;;
    c2) A="--batch 1" ;;
    c5) A="--batch 4 --res 768" ;;
    *) echo "unknown config $cfg"; exit 1 ;;
  esac
  P=/tmp/prof_$cfg; rm -rf $P; mkdir -p $P
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o k -- python3 -u bench.py $A --steps 1 --warmup 1 \
    --no-cpu-baseline --no-pmc --no-configs > gpurun_out/prof/${cfg}_stdout.log 2> gpurun_out/prof/${cfg}_stderr.log \
    || { echo "$cfg trace rc $?"; tail -20 gpurun_out/prof/${cfg}_stderr.log; exit 1; }
  kt=$(find $P -name "*kernel_trace.csv" | head -1)
  cp $(find $P -name "*kernel_stats.csv" | head -1) gpurun_out/prof/${cfg}_kernel_stats.csv
  python3 scripts/kt_summary.py $kt 2 > gpurun_out/prof/${cfg}_by_kernel.txt
  gzip -c $kt > gpurun_out/prof/${cfg}_kernel_trace.csv.gz
  head -16 gpurun_out/prof/${cfg}_by_kernel.txt
done
if [ -n "$LEDGER" ]; then
  timeout -k 10 240 python3 -u scripts/ledger.py --batch 8 --out gpurun_out/prof/ledger_c3.txt > gpurun_out/prof/ledger_c3.log 2>&1 \
    && timeout -k 10 240 python3 -u scripts/ledger.py --batch 1 --out gpurun_out/prof/ledger_c2.txt > gpurun_out/prof/ledger_c2.log 2>&1 \
    || { echo "ledger failed"; exit 1; }
  head -14 gpurun_out/prof/ledger_c3.txt gpurun_out/prof/ledger_c2.txt
fi

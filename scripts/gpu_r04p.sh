#!/bin/bash
# Round 4: in-launch split-K combine read-back budget A/B at small budgets (0 = off), same box,
# and a c2 kernel trace at the 704 KiB budget (which convs lose).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
for r in 1 2; do
  for kb in 0 96 200; do
    C2D_SPLITK_TAIL_KB=$kb timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail_kb $kb round $r: c3', d['value'], 'c2', d['c2_latency_s'], 'c5', d['c5_images_per_s'])" | tee -a $O/ab.txt || exit 1
  done
done
P=/tmp/prof; rm -rf $P; mkdir -p $P
C2D_SPLITK_TAIL_KB=704 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c2_stdout.log 2> $O/c2_stderr.log || { echo "c2 prof rc $?"; tail -5 $O/c2_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c2 -name "*kernel_trace.csv" | head -1) 2 > $O/c2_by_kernel_704.txt
head -40 $O/c2_by_kernel_704.txt

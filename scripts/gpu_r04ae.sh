#!/bin/bash
# Round 4: which ops issue the ~15 small device copies per denoise step (c2 kernel trace, dispatch order).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > /tmp/c2.log 2>&1 || { echo "prof rc $?"; tail -5 /tmp/c2.log; exit 1; }
python3 scripts/kt_neighbours.py $(find $P/c2 -name "*kernel_trace.csv" | head -1) copyBuffer

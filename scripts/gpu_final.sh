#!/bin/bash
# Round evidence on one box: the default bench line (PMC traffic passes, c1 CPU leg, c2 / c5 / c1-GPU side
# configs), the dominant-kernel and d = 40 attention rocprofv3 --stats + PMC counter passes, then rocprofv3
# kernel traces of c3 / c2 / c5 and the c3 / c2 step ledgers.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -5 gpurun_out/bench_final.err; exit 1; }
tail -3 gpurun_out/bench_final.err; cat gpurun_out/bench_final.json
bash scripts/gpu_profiles.sh || exit $?
NOBENCH=1 TRACES="${TRACES-c3 c2 c5}" LEDGER=1 bash scripts/gpu_bench_prof.sh

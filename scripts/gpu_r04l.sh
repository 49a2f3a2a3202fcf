#!/bin/bash
# Round 4 evidence, part 1: the whole -m gpu suite on the current tree (parity metrics TSV kept).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
rm -f gpurun_out/parity_metrics.tsv
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/pytest_gpu.txt; cp gpurun_out/parity_metrics.tsv $O/ 2>/dev/null
exit $rc

#!/bin/bash
# Round 4: end-to-end tests after the oracle's projector restatement (oracle/projectors_ref.py), and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
rm -f gpurun_out/parity_metrics.tsv
timeout -k 10 900 python -u -m pytest tests/test_pipeline_gpu.py tests/test_golden_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/pytest.log; cp gpurun_out/parity_metrics.tsv $O/ 2>/dev/null; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 $O/smoke.log; exit $rc

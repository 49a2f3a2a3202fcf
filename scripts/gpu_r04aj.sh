#!/bin/bash
# Round 4: tail-split parity -- the kernel tests and the c5-shape pipeline test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -k "not graph_replay_is_repeatable or c5" > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; exit $rc

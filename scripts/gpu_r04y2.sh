#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for z in 0 1 2; do echo "== C2D_GN_ZERO=$z"; C2D_GN_ZERO=$z timeout -k 10 120 python -u scripts/gn_graph_diag.py 2>&1 | grep -v amdgpu || exit 1; done

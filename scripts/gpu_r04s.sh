#!/bin/bash
# Round 4: deep-ring DMA tile variants (4 = 64x64 x 6 stages, 5 = 128x128 x 4, 6 = 128x160 x 3,
# 10 = 64x160 x 4) for the latency-bound N = 2 (c2) shapes: forced-tile tests, then graph-replayed
# plan sweeps at batch 1 against the current tiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "every_dma_tile or epilogue_operand" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/sweep_tiles_graph.py --batch 1 --only "1x1" --tiles 3,4,2,5,9,10,8,6 --splits 1,2,4,8 > $O/sweep_b1_1x1.txt 2>&1 || { tail -5 $O/sweep_b1_1x1.txt; exit 1; }
timeout -k 10 500 python -u scripts/sweep_tiles_graph.py --batch 1 --only "qkv" --tiles 3,4,2,5,9,10,8,6 --splits 1,2,4 > $O/sweep_b1_qkv.txt 2>&1 || { tail -5 $O/sweep_b1_qkv.txt; exit 1; }
timeout -k 10 600 python -u scripts/sweep_tiles_graph.py --batch 1 --only "3x3" --tiles 7,3,4,9,10,6,2,5 --splits 2,4,6,8,12,16 > $O/sweep_b1_3x3.txt 2>&1 || { tail -5 $O/sweep_b1_3x3.txt; exit 1; }
echo sweeps done

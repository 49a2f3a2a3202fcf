#!/bin/bash
# Round 4: in-launch split-K combine (ticketed last slice) -- kernel tests (bit-identity with the
# two-launch form, replay / uneven-load repeatability, every forced tile and split count), the
# UNet-vs-oracle tests, then a same-box bench A/B of the read-back budget (0 = off).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py -k "in_launch or split_k or every_dma_tile or padded_source or epilogue_operand" -x -v --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1
rc=$?; echo "pytest kernels exit $rc"; tail -3 $O/pytest_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_unet_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_u.log 2>&1
rc=$?; echo "pytest unet exit $rc"; tail -3 $O/pytest_u.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for kb in 0 704 1400; do
    C2D_SPLITK_TAIL_KB=$kb timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail_kb $kb round $r: c3', d['value'], 'c2', d['c2_latency_s'], 'c5', d['c5_images_per_s'])" | tee -a $O/ab.txt || exit 1
  done
done

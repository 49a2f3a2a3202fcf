# row-ring tiles: parity tests, then per-shape A/B (scripts/rowring_ab.py) for each library in LIBS
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-padded_source or every_dma_tile_forced}" > gpurun_out/rr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rr_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in ${LIBS:-libc2d_hip}; do
  echo "== $lib"
  C2D_LIB=$PWD/clap2diffusion_amd/$lib.so timeout -k 10 300 python -u scripts/rowring_ab.py $RR_ARGS > gpurun_out/rr_ab_$lib.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/rr_ab_$lib.txt; [ $rc -eq 0 ] || exit $rc
done
for lib in ${LIBS2}; do
  echo "== $lib (c2)"
  C2D_LIB=$PWD/clap2diffusion_amd/$lib.so timeout -k 10 300 python -u scripts/rowring_ab.py --batch 1 > gpurun_out/rr_ab_c2_$lib.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/rr_ab_c2_$lib.txt; [ $rc -eq 0 ] || exit $rc
done
for bt in ${SWEEP}; do
  timeout -k 10 500 python -u scripts/rr_sweep.py --batch $bt > gpurun_out/rr_sweep_b$bt.txt 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/rr_sweep_b$bt.txt | grep -v "^  N="; [ $rc -eq 0 ] || exit $rc
done

# attention parity + A/B per library (ATTN_LIBS), row-ring tests incl. tile 45, level-2 sweeps, the bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for lib in ${ATTN_LIBS}; do
  C2D_LIB=$PWD/clap2diffusion_amd/$lib.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k attention > gpurun_out/attn_tests_$lib.log 2>&1
  echo "== $lib attention tests rc $?: $(tail -1 gpurun_out/attn_tests_$lib.log)"
done
for r in 1 2; do for lib in ${ATTN_LIBS}; do
  echo "== attention timing $lib"
  C2D_LIB=$PWD/clap2diffusion_amd/$lib.so timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -E "d80|d40" | grep -v amdgpu.ids || exit 1
done; done
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "padded_source or every_dma_tile" > gpurun_out/rr3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rr3_tests.log; [ $rc -eq 0 ] || exit $rc
for bt in 8 1; do
  timeout -k 10 400 python -u scripts/rr_sweep.py --batch $bt --only-h 16 > gpurun_out/rr_sweep45_b$bt.txt 2>&1 || exit 1
  grep -E "^(WIN|keep|    )" gpurun_out/rr_sweep45_b$bt.txt
done

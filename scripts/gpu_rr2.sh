# UNet / pipeline / attention parity with the current library, the prefix sweeps, attention A/B, then the bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-padded_source or unet or pipeline or attention}" > gpurun_out/rr2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rr2_tests.log; [ $rc -eq 0 ] || exit $rc
for bt in 1 8; do
  timeout -k 10 200 python -u scripts/rr_sweep.py --prefix --batch $bt > gpurun_out/rr_sweep_prefix_b$bt.txt 2>&1 || exit 1
  grep -E "^(WIN|keep|    )" gpurun_out/rr_sweep_prefix_b$bt.txt
done
for lib in ${ATTN_LIBS}; do
  echo "== attention $lib"
  C2D_LIB=$PWD/clap2diffusion_amd/$lib.so timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc

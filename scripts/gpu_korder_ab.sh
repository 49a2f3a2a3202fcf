cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv or gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for ko in 0 1; do echo "== korder $ko"; C2D_GEMM_KORDER=$ko ONLY=conv timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v amdgpu || exit 1; done
for ko in 0 1; do C2D_GEMM_KORDER=$ko timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf$ko -o f -- python3 -u scripts/roof_kernel.py 5 > gpurun_out/pf$ko.log 2>&1 || exit 1; f=$(find /tmp/pf$ko -name "*counter_collection.csv"); python3 -c "
import csv,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if 'igemm' in r['Kernel_Name']]
print('korder $ko FETCH_SIZE KiB per launch', v[-3:])"; done

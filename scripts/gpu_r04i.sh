#!/bin/bash
# Round 4: cache policy of the persistent GEGLU kernel's carried-epilogue stores (plain / nt / sc1):
# L0 / L1 GEGLU timings, same box, two alternations, then FETCH_SIZE / WRITE_SIZE per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
L=$PWD/clap2diffusion_amd
for r in 1 2; do
  for v in "" _nt _sc1; do
    echo "== lib libc2d_hip$v.so round $r"
    C2D_LIB=$L/libc2d_hip$v.so timeout -k 10 120 python -u scripts/ab_tiles.py --shapes geglu0,geglu1 --plans 0 --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt
cat $O/ab.txt
for v in "" _nt _sc1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    C2D_LIB=$L/libc2d_hip$v.so timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmc_$v$ctr -o p -- python3 -u scripts/one_gemm.py 1 64 320 2560 6 --geglu > /dev/null 2>&1 || { echo "pmc $v $ctr failed"; exit 1; }
    f=$(find /tmp/pmc_$v$ctr -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$v" "$ctr" <<'PY'
import csv, sys
v = sorted(float(r['Counter_Value']) for r in csv.DictReader(open(sys.argv[1])) if 'igemm' in r['Kernel_Name'])
print(f"lib{sys.argv[2] or '(plain)'} {sys.argv[3]} median {v[len(v)//2]:.0f} KiB")
PY
  done
done | tee $O/pmc.txt

#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, --pmc only) over single-kernel drivers:
# NAMES="conv attn" (conv: scripts/roof_kernel.py, attn: scripts/roof_attn.py); per pass the
# per-dispatch counter CSV is summarised (median over dispatches of the named kernel) into
# gpurun_out/pmc/<name>_counters.txt and the raw CSVs are kept.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
G3="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"
for name in ${NAMES:-conv attn}; do
  unset C2D_GEMM_TILE
  case $name in
    conv[0-9]*) export C2D_GEMM_TILE=${name#conv}; PROG="python3 -u scripts/roof_kernel.py 5"; FILT=igemm ;;
    conv*) PROG="python3 -u scripts/roof_kernel.py 5"; FILT=igemm ;;
    attn9216) PROG="python3 -u scripts/roof_attn.py 5 9216 8"; FILT=attn ;;
    attn*) PROG="python3 -u scripts/roof_attn.py 5"; FILT=attn ;;
  esac
  i=0
  : > gpurun_out/pmc/${name}_counters.txt
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${name}_$i -o p -- $PROG > gpurun_out/pmc/${name}_run$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 gpurun_out/pmc/${name}_run$i.log; exit 1; }
    f=$(find /tmp/pmc_${name}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" gpurun_out/pmc/${name}_pass$i.csv
    python3 - "$f" "$FILT" >> gpurun_out/pmc/${name}_counters.txt <<'PY'
import csv, sys, collections
f, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if filt in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for c, v in sorted(agg.items()):
    v.sort()
    print(f"{c:28s} {v[len(v)//2]:18.1f}  (median of {len(v)} dispatches)")
PY
  done
  echo "== $name"; cat gpurun_out/pmc/${name}_counters.txt
done

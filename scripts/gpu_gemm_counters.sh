#!/bin/bash
# rocprofv3 over single-GEMM drivers of the transformer-block projections (N = 16, 64^2 latents):
# a kernel-trace pass (average duration) and five --pmc passes (one counter group each: SQ issue /
# MFMA, LDS, VALU + L2, FETCH_SIZE, WRITE_SIZE), summarised per shape into gpurun_out/gemmpmc/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/gemmpmc${TAG}; mkdir -p $D   # TAG: a suffix per run (e.g. the forced tile, C2D_GEMM_TILE)
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
G3="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
for name in ${NAMES:-geglu0 qkv0 res0 l2res}; do
  case $name in
    geglu0) ARGS="1 64 320 2560 6 --geglu" ;;
    qkv0) ARGS="1 64 320 960 6" ;;
    res0) ARGS="1 64 320 320 6 --res" ;;
    l2res) ARGS="1 16 1280 1280 6 --res" ;;
    conv0) ARGS="3 64 320 320 6 --res" ;;
    conv0p) ARGS="3 64 320 320 6 --res --pad" ;;
  esac
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$name -o k -- python3 -u scripts/one_gemm.py $ARGS > $D/${name}_kt.log 2>&1 || { echo "$name kt failed"; tail -5 $D/${name}_kt.log; exit 1; }
  cp $(find /tmp/kt_$name -name "*kernel_stats.csv" | head -1) $D/${name}_kernel_stats.csv
  i=0; : > $D/${name}_counters.txt
  for grp in "$G1" "$G2" "$G3" "$G4" "$G5"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${name}_$i -o p -- python3 -u scripts/one_gemm.py $ARGS > $D/${name}_run$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $D/${name}_run$i.log; exit 1; }
    f=$(find /tmp/pmc_${name}_$i -name "*counter_collection.csv" | head -1)
    python3 - "$f" >> $D/${name}_counters.txt <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'igemm' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for c, v in sorted(agg.items()):
    v.sort()
    print(f"{c:28s} {v[len(v)//2]:18.1f}  (median of {len(v)} dispatches)")
PY
  done
  echo "== $name"; cat $D/${name}_counters.txt; grep -h igemm $D/${name}_kernel_stats.csv | cut -c1-160
done

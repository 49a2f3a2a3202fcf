#!/bin/bash
# Same-box A/B of variants, alternated ROUNDS times (default 2) so drift between boxes and over a run
# cancels.  A variant is "label:VAR=val,VAR2=val" (environment for that arm; C2D_LIB=<path> selects
# another build of libc2d_hip.so, PYROOT=<dir> another Python tree with its own bench.py).
#   VARIANTS="fold0:C2D_FOLD_FF_OUT=0 fold1:C2D_FOLD_FF_OUT=1" bash scripts/gpu_ab.sh
# The library reads no environment: a kernel-side candidate is a variant build made here first
#   python -m clap2diffusion_amd.build --variant gn0 --define C2D_TUNE_GN_FOLD=0
#   VARIANTS="base:C2D_LIB=clap2diffusion_amd/libc2d_hip.so gn0:C2D_LIB=clap2diffusion_amd/libc2d_hip_gn0.so"
#   CMD=norm   each arm runs scripts/bench_norm_graph.py (graph-replayed GN / LN shapes)
#   CMD=shapes each arm runs scripts/unet_shapes.py (per-shape GEMM breakdown)
#   CMD=attn   each arm runs scripts/bench_attn.py (the UNet attention shapes, random operands)
#   CMD=bench  (default) the bench line with BENCH_ARGS (default: short, no CPU / PMC / configs)
# PYTEST_K (optional): run that -m gpu subset once per arm first.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BENCH_ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-configs}
arm() {  # label, comma-separated env, command...
  local label=$1 envs=$2; shift 2
  (
    root=.
    for kv in ${envs//,/ }; do
      case $kv in PYROOT=*) root=${kv#PYROOT=} ;; C2D_LIB=*) export C2D_LIB=$PWD/${kv#C2D_LIB=} ;; *) export "$kv" ;; esac
    done
    cd "$root" && "$@"
  )
}
for v in $VARIANTS; do
  [ -z "$PYTEST_K" ] && break
  label=${v%%:*}; envs=${v#*:}
  arm "$label" "$envs" timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "$PYTEST_K" > gpurun_out/ab/pytest_$label.log 2>&1
  rc=$?; echo "== $label pytest: $(tail -1 gpurun_out/ab/pytest_$label.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    label=${v%%:*}; envs=${v#*:}
    echo "== $label (round $r)"
    case ${CMD:-bench} in
      norm) arm "$label" "$envs" timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep -E "^(GN|LN)" || exit 1 ;;
      attn) arm "$label" "$envs" timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v "amdgpu.ids\|^\[W" || exit 1 ;;
      shapes) arm "$label" "$envs" timeout -k 10 300 python -u scripts/unet_shapes.py 2>&1 | grep -v "amdgpu.ids\|^\[W" \
                | sed -n "1,${SHAPES_LINES:-24}p" || exit 1 ;;
      bench) arm "$label" "$envs" timeout -k 10 400 python -u bench.py $BENCH_ARGS > gpurun_out/ab/${label}_$r.json \
               2> gpurun_out/ab/${label}_$r.err || { tail -5 gpurun_out/ab/${label}_$r.err; exit 1; }
             python3 - gpurun_out/ab/${label}_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = [f"c3 {d['value']:.4f} img/s", f"dominant {d['roofline']['avg_us']} us"]
if "c2_latency_s" in d:
    x += [f"c2 {d['c2_latency_s']} s", f"c5 {d['c5_images_per_s']} img/s"]
print("  ".join(x))
PY
             ;;
    esac
  done
done

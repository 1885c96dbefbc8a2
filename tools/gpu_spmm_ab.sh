#!/bin/bash
# SpMM halves A/B: the in-tree library vs tools/bin/libhnm_<variant>.so (timing per half,
# 3-layer forward() rows compared, the variant's LightGCN GPU tests, FETCH_SIZE/TCC per half).
#   bash tools/gpu_spmm_ab.sh <tag> <variant>
set -uo pipefail
TAG=$1; VAR=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
VLIB="$ROOT/tools/bin/libhnm_$VAR.so"
run() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "$name failed"; tail -20 "$OUT/$name.err"; exit 1; }
  tail -4 "$OUT/$name.out"; }
run base64 240 python tools/spmm_halves.py --d 64 --dump "$OUT/base64.npz"
run var64 240 env HNM_LIB_PATH="$VLIB" python tools/spmm_halves.py --d 64 --dump "$OUT/var64.npz"
run base128 240 python tools/spmm_halves.py --d 128
run var128 240 env HNM_LIB_PATH="$VLIB" python tools/spmm_halves.py --d 128
run cmp 60 python -c "
import numpy as np
a=np.load('$OUT/base64.npz'); b=np.load('$OUT/var64.npz')
for k in ('fu','fi'):
    s=np.abs(a[k]).max(); print(k, 'max |diff|/scale', float(np.abs(a[k]-b[k]).max()/s))
    assert np.abs(a[k]-b[k]).max() <= 1e-5*s"
run vtests 600 env HNM_LIB_PATH="$VLIB" python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "lightgcn or propagat or history"
cd /tmp && export TMPDIR=/tmp
i=0
for lib in base var; do for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  if [ $lib = var ]; then export HNM_LIB_PATH="$VLIB"; else unset HNM_LIB_PATH; fi
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_${lib}_$i" -o run -- python3 "$ROOT/tools/spmm_halves.py" --d 64 --reps 2 > "$OUT/pmc_${lib}_$i.log" 2>&1 || { echo "pmc $lib $i failed"; tail -5 "$OUT/pmc_${lib}_$i.log"; exit 1; }
done; done
unset HNM_LIB_PATH
echo ok

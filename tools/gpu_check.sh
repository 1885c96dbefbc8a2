#!/bin/bash
# GPU session: parity tests + smoke() + default bench (all workloads) + 2-rank launcher
# rehearsal (gloo on one GPU).
#   bash tools/gpu_check.sh <tag> [pytest -k expr]   (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=${1:-r}
KEXPR=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 "$OUT/$name.out"; tail -20 "$OUT/$name.err"; exit $rc; fi
  tail -3 "$OUT/$name.out"
}
if [ -n "$KEXPR" ]; then
  step tests 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread -k "$KEXPR"
else
  step tests 1000 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_ncf 900 python bench.py
export HNM_DIST_BACKEND=gloo
step bench_2rank 400 python bench.py --gpus 2 --workload lightgcn128 --steps 5 --warmup 2
echo ok

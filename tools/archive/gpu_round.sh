#!/bin/bash
# One GPU session: parity tests, every bench workload, rocprofv3 kernel stats per workload.
#   bash tools/gpu_round.sh <tag>      (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=${1:-r}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -20 "$OUT/$name.err"; exit $rc; fi
}
step tests 900 python -m pytest tests -x -q -m gpu
step bench_ncf 300 python bench.py
step bench_lightgcn 400 python bench.py --workload lightgcn --no-cpu-baseline
step bench_lightgcn128 400 python bench.py --workload lightgcn128 --no-cpu-baseline
step bench_mf 300 python bench.py --workload mf --no-cpu-baseline
step bench_widedeep 600 python bench.py --workload widedeep --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
for w in ncf lightgcn widedeep; do
  extra="--steps 5 --warmup 2"
  [ $w = widedeep ] && extra="--steps 3 --warmup 1"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- \
    python3 "$ROOT/bench.py" --workload $w $extra --no-cpu-baseline > "$OUT/prof_$w.log" 2>&1 \
    || { echo "rocprof $w failed"; exit 1; }
done
echo ok

#!/bin/bash
# Full GPU session: parity tests, the default bench line (NCF headline + every other workload
# + B=1 serve latencies, as the driver runs it), personalised NCF weights, the 2-rank
# launcher rehearsal, and optional rocprofv3 kernel stats per workload.
#   bash tools/gpu_full.sh <tag> [prof]     (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=${1:-r}
PROF=${2:-}
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
  tail -c 600 "$OUT/$name.out"; echo
}
step tests 1000 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread
step bench_default 900 python bench.py
step bench_ncf_personal 300 python bench.py --weights personal --no-cpu-baseline
HNM_DIST_BACKEND=gloo step bench_2rank 400 python bench.py --gpus 2 --workload lightgcn128 --steps 5 --warmup 2
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  for w in ncf lightgcn widedeep mf ncf_deep; do
    extra=""  # the bench defaults, so the averages match the bench line's HIP-event timing
    [ $w = widedeep ] && extra="--steps 3 --warmup 1"
    echo "== prof $w $(date +%T)"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- \
      python3 "$ROOT/bench.py" --workload $w $extra --profile-only > "$OUT/prof_$w.log" 2>&1 \
      || { echo "rocprof $w failed"; exit 1; }
  done
fi
echo ok

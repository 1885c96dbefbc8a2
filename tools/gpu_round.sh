#!/bin/bash
# Round-end GPU session on the in-tree build: the full -m gpu suite, smoke(), the default bench
# line (every workload + serve latencies, as the driver runs it), rocprofv3 kernel stats per
# workload over `--profile-only`, PMC passes for the given workloads, a 2-rank gloo rehearsal.
#   bash tools/gpu_round.sh <tag> [pmc workloads...]      (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=${1:-r}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
step() {  # name timeout cmd...   (stops the session on anything but success / test failures)
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then echo "step $name rc=$rc"; tail -25 "$OUT/$name.out"; tail -10 "$OUT/$name.err"; fi
  [ $rc -eq 0 ] || [ "$name" = tests -a $rc -eq 1 ] || exit $rc
  tail -c 400 "$OUT/$name.out"; echo
}
step tests 1100 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 900 python bench.py
HNM_DIST_BACKEND=gloo step bench_2rank 400 python bench.py --gpus 2 --workload lightgcn128 --steps 5 --warmup 2
cd /tmp && export TMPDIR=/tmp
for w in ncf lightgcn lightgcn128 widedeep mf; do
  extra=""
  [ $w = widedeep ] && extra="--steps 3 --warmup 1"
  echo "== prof $w $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- \
    python3 "$ROOT/bench.py" --workload $w $extra --profile-only > "$OUT/prof_$w.log" 2>&1 \
    || { echo "rocprof $w failed"; tail -5 "$OUT/prof_$w.log"; exit 1; }
done
cd "$ROOT"
for w in "$@"; do
  bash tools/pmc_profile.sh $w gpurun_out/${TAG}_pmc_$w || exit 1
done
echo ok

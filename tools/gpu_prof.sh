#!/bin/bash
# rocprofv3 kernel stats per workload (the bench defaults, --profile-only) and the LightGCN PMC
# passes, outputs under gpurun_out/<tag>/ and gpurun_out/<tag>_pmc_<w>/.
#   bash tools/gpu_prof.sh <tag> [pmc workloads...]
set -uo pipefail
TAG=${1:-r}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for w in "$@"; do
  bash tools/pmc_profile.sh $w gpurun_out/${TAG}_pmc_$w || exit 1
done
cd /tmp && export TMPDIR=/tmp
for w in ncf lightgcn lightgcn128 widedeep mf; do
  extra=""
  [ $w = widedeep ] && extra="--steps 3 --warmup 1"
  echo "== prof $w $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- \
    python3 "$ROOT/bench.py" --workload $w $extra --profile-only > "$OUT/prof_$w.log" 2>&1 \
    || { echo "rocprof $w failed"; tail -5 "$OUT/prof_$w.log"; exit 1; }
done
echo ok

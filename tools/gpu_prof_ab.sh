#!/bin/bash
# rocprofv3 kernel stats of `bench.py --workload <w> --profile-only` for variant libraries, and
# FETCH_SIZE / TCC hit-miss passes for the first variant.
#   bash tools/gpu_prof_ab.sh <tag> <workload> variants...
set -uo pipefail
TAG=$1; W=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  export HNM_LIB_PATH=$ROOT/tools/bin/libhnm_$t.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$t" -o $W -- \
    python3 "$ROOT/bench.py" --workload $W --profile-only > "$OUT/prof_$t.log" 2>&1 || { echo "prof $t failed"; tail -5 "$OUT/prof_$t.log"; exit 1; }
  f=$(ls "$OUT"/prof_$t/*kernel_stats.csv | head -1)
  echo "== $t"; cut -d, -f1-4 "$f" | head -8 | cut -c1-160
done
i=0
for t in "$@"; do
  export HNM_LIB_PATH=$ROOT/tools/bin/libhnm_$t.so
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_$t/p$i" -o run -- python3 "$ROOT/bench.py" --workload $W --steps 2 --warmup 1 --profile-only > "$OUT/pmc_${t}_$i.log" 2>&1 || { echo "pmc $t $i failed"; tail -5 "$OUT/pmc_${t}_$i.log"; exit 1; }
  done
done
echo ok

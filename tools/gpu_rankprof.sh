#!/bin/bash
# rocprofv3 kernel stats of tools/rank_shape_probe.py at one world size (the per-rank work of the
# item-sharded step on one GPU), top kernels by total time with their average duration.
#   bash tools/gpu_rankprof.sh <tag> <ncf|mf> <W> [modes]     (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=$1; WL=$2; W=$3; MODES=${4:-lists}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG/${WL}_w$W"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/tools/rank_shape_probe.py" "$WL" "$W" "$MODES" > "$OUT/probe.out" 2> "$OUT/probe.err" \
  || { echo "rocprof failed"; tail -5 "$OUT/probe.err"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  n={r["Calls"]:>5}  avg={float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
grep "W=" "$OUT/probe.out"

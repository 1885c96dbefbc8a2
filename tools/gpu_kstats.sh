#!/bin/bash
# rocprofv3 kernel stats of one bench.py invocation (--profile-only added), top kernels printed.
#   bash tools/gpu_kstats.sh <tag> <bench args...>      (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" "$@" --profile-only > "$OUT/bench.out" 2> "$OUT/bench.err" \
  || { echo "rocprof failed"; tail -5 "$OUT/bench.err"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms  n={r["Calls"]:>5}  avg={float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
tail -c 300 "$OUT/bench.out"

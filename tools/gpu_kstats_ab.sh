#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of variant libraries
# (tools/bin/libhnm_<tag>.so via HNM_LIB_PATH) on one bench workload.
#   bash tools/gpu_kstats_ab.sh <outtag> <workload> "<kernel regex>" "<bench args>" tag1 tag2 ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$1; W=$2; PAT=$3; ARGS=$4; shift 4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  HNM_LIB_PATH=$ROOT/tools/bin/libhnm_$t.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$t -o k -- python3 $ROOT/bench.py --workload $W $ARGS --no-cpu-baseline --no-extras > $OUT/$t.log 2>&1 || { echo "variant $t failed"; tail -5 $OUT/$t.log; exit 1; }
  f=$(find $OUT/$t -name 'k_kernel_stats.csv' | head -1)
  python3 - "$f" "$PAT" "$t" <<'PY'
import csv, re, sys
f, pat, tag = sys.argv[1:4]
for r in csv.DictReader(open(f)):
    if re.search(pat, r["Name"]):
        print(tag, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
done

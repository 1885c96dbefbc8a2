#!/bin/bash
# GPU check after a kernel change: every GPU test, chosen bench workloads, and rocprofv3
# per-kernel averages of the in-tree library on each workload.
#   bash tools/gpu_step.sh <tag> "<workload ...>" ["<kernel regex>"]
set -uo pipefail
TAG=${1:-s}; WLS=${2:-ncf}; PAT=${3:-.}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $OUT/tests.out 2>&1 || { grep -E "FAILED|Error" $OUT/tests.out | head; tail -30 $OUT/tests.out; exit 1; }
tail -1 $OUT/tests.out
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-extras > $OUT/bench_$w.out 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$w.out').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d.get('prefilter'))"
done
cd /tmp && export TMPDIR=/tmp
for w in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$w -o k -- python3 $ROOT/bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $OUT/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 $OUT/prof_$w.log; exit 1; }
  f=$(find $OUT/prof_$w -name 'k_kernel_stats.csv' | head -1)
  python3 - "$f" "$PAT" "$w" <<'PY'
import csv, re, sys
f, pat, tag = sys.argv[1:4]
for r in csv.DictReader(open(f)):
    if re.search(pat, r["Name"]):
        print(tag, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["MinNs"]) / 1e3, 2))
PY
done
echo ok

#!/bin/bash
# Quick GPU check: scan timing harness, a pytest -k selection, then chosen bench workloads.
#   bash tools/gpu_quick.sh <tag> "<pytest -k expr>" "<workload ...>"
set -uo pipefail
TAG=${1:-q}; KEXPR=${2:-}; WLS=${3:-ncf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -x tools/bin/scan_ablation ]; then
  timeout -k 10 60 tools/bin/scan_ablation > $OUT/scan_timing.txt 2>&1 || { cat $OUT/scan_timing.txt; exit 1; }
  cat $OUT/scan_timing.txt
fi
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread -k "$KEXPR" > $OUT/tests.out 2>&1 || { grep -E "FAILED|Error" $OUT/tests.out | head; tail -30 $OUT/tests.out; exit 1; }
  tail -1 $OUT/tests.out
fi
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.out 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$w.out').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d.get('prefilter'))"
done

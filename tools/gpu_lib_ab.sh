#!/bin/bash
# A/B bench of variant libraries (tools/bin/libhnm_<tag>.so via HNM_LIB_PATH) on one workload,
# after the in-tree library's parity tests selected by -k.
#   bash tools/gpu_lib_ab.sh <outtag> <pytest -k expr|-> <workload> "<bench args>" tag1 tag2 ...
set -uo pipefail
OUT=gpurun_out/$1; K=$2; W=$3; ARGS=$4; shift 4
mkdir -p $OUT
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 180 --timeout-method thread > $OUT/tests.out 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.out; exit 1; }
  tail -3 $OUT/tests.out
fi
for t in "$@"; do
  HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 300 python bench.py --workload $W $ARGS --no-cpu-baseline --no-extras > $OUT/${W}_$t.out 2> $OUT/${W}_$t.err || { echo "variant $t failed"; tail -5 $OUT/${W}_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${W}_$t.out').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['roofline']['frac'])"
done

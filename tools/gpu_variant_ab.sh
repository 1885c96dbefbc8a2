#!/bin/bash
# round-4 A/B: GPU tests (-k filter) on the in-tree build, then bench lines of the workloads in
# $WORKLOADS (default: lightgcn lightgcn128) for each variant library (tools/bin/libhnm_<tag>.so)
set -uo pipefail
OUT=gpurun_out/$1; K=$2; shift 2
mkdir -p $OUT
if [ "$K" = "all" ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1
  echo "tests rc=$?"; grep -E "FAILED|ERROR" $OUT/tests.out | head -30; tail -3 $OUT/tests.out
elif [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $OUT/tests.out | head -20; tail -40 $OUT/tests.out; exit 1; }
  tail -3 $OUT/tests.out
fi
for W in ${WORKLOADS:-lightgcn lightgcn128}; do
for t in "$@"; do
  HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --no-extras --profile-only > $OUT/${W}_$t.out 2> $OUT/${W}_$t.err || { echo "variant $t failed"; tail -5 $OUT/${W}_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${W}_$t.out').read().strip().splitlines()[-1]); print('$W $t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['roofline']['frac'])"
done; done

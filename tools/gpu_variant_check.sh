#!/bin/bash
# Parity tests (pytest -k selection) run AGAINST a variant library, then an A/B bench of the
# product build and the variants on one workload.
#   bash tools/gpu_variant_check.sh <outtag> "<pytest -k expr>" <workload> "<bench args>" tag1 [tag2 ...]
# (the first tag's library is the one tested; "prod" = the in-tree build)
set -uo pipefail
OUT=gpurun_out/$1; K=$2; W=$3; ARGS=$4; shift 4
mkdir -p $OUT
lib() { [ "$1" = prod ] && echo "$PWD/hnm_recommendation_amd/libhnm_mi355x.so" || echo "$PWD/tools/bin/libhnm_$1.so"; }
HNM_LIB_PATH=$(lib $1) timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 180 --timeout-method thread > $OUT/tests_$1.out 2>&1 || { echo "tests failed ($1)"; grep -E "FAILED|Error" $OUT/tests_$1.out | head; tail -30 $OUT/tests_$1.out; exit 1; }
tail -1 $OUT/tests_$1.out
for t in prod "$@"; do
  HNM_LIB_PATH=$(lib $t) timeout -k 10 300 python bench.py --workload $W $ARGS --no-cpu-baseline --no-extras > $OUT/${W}_$t.out 2> $OUT/${W}_$t.err || { echo "variant $t failed"; tail -5 $OUT/${W}_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${W}_$t.out').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['roofline']['frac'], d.get('prefilter'))"
done

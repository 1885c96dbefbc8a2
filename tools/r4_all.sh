#!/bin/bash
# round-4 GPU session: full -m gpu suite, SpMM short-walk A/B (d=64, d=128), W&D x_lo A/B.
#   bash tools/r4_all.sh <tag> "<spmm variants>" "<wd variants>"
set -uo pipefail
TAG=$1; SV=$2; WV=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" $OUT/tests.out | head -30; tail -2 $OUT/tests.out
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (reported above); anything else: stop
ab() {  # workload extra-args variants...
  local W=$1 X=$2; shift 2
  for t in "$@"; do
    HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 300 python bench.py --workload $W $X --no-cpu-baseline --no-extras --profile-only > $OUT/${W}_$t.out 2> $OUT/${W}_$t.err || { echo "variant $t failed"; tail -5 $OUT/${W}_$t.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${W}_$t.out').read().strip().splitlines()[-1]); print('$W $t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['roofline']['frac'], d.get('prefilter'))"
  done
}
ab lightgcn "" $SV
ab lightgcn128 "" $SV
if [ -n "$WV" ]; then
  ab widedeep "--steps 3 --warmup 1" $WV
  for t in $WV; do
    HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "wd_ or widedeep" --timeout 300 --timeout-method thread > $OUT/wdtests_$t.out 2>&1; echo "wd tests $t rc=$?"; tail -1 $OUT/wdtests_$t.out
  done
fi
echo ok

#!/bin/bash
# W&D certified path: parity + prefilter tests, bench (certified and exact), kernel stats.
set -uo pipefail
OUT=gpurun_out/${1:-wd}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_prefilter.py -k "wd_" -rP > $OUT/tests_wd.log 2>&1 || { echo "wd tests failed"; tail -40 $OUT/tests_wd.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "widedeep or wd" > $OUT/tests_wdpar.log 2>&1 || { echo "wd parity failed"; tail -40 $OUT/tests_wdpar.log; exit 1; }
timeout -k 10 300 python bench.py --workload widedeep --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_wd.json 2> $OUT/bench_wd.err || { echo "bench failed"; tail -20 $OUT/bench_wd.err; exit 1; }
cat $OUT/bench_wd.json
grep -E "W&D" $OUT/tests_wd.log || true

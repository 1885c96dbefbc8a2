#!/bin/bash
# LightGCN restricted propagation + SpMM finish rewrite + small-batch row top-K: tests, benches.
set -uo pipefail
OUT=gpurun_out/r2c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread \
  -k "lightgcn or row_topk or sharding or golden" > $OUT/tests.out 2>&1 || { tail -40 $OUT/tests.out; exit 1; }
tail -2 $OUT/tests.out
for w in lightgcn lightgcn128; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.out 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  tail -1 $OUT/bench_$w.out
done
timeout -k 10 300 python bench.py --latency --steps 200 > $OUT/lat_ncf.out 2> $OUT/lat_ncf.err && cat $OUT/lat_ncf.out

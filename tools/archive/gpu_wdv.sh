#!/bin/bash
# A/B timing of W&D scan variant libraries (tools/bin/libhnm_wd<tag>.so) with the bench.
set -uo pipefail
OUT=gpurun_out/${1:-wdv}; shift
mkdir -p $OUT
for t in "$@"; do
  HNM_LIB_PATH=$PWD/tools/bin/libhnm_wd$t.so timeout -k 10 300 python bench.py --workload widedeep --steps 3 --warmup 1 --no-cpu-baseline > $OUT/wd_$t.out 2> $OUT/wd_$t.err || { echo "variant $t failed"; tail -5 $OUT/wd_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/wd_$t.out').read().strip().splitlines()[-1]); print('$t', d['value'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['prefilter']['candidates_per_row'])"
done

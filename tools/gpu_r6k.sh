set -uo pipefail
OUT=gpurun_out/r6k; mkdir -p $OUT
run() {  # weights variants...
  local wt=$1; shift
  for t in "$@"; do
    HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 300 python bench.py --workload ncf --weights $wt --profile-only > $OUT/ncf_${wt}_$t.out 2> $OUT/ncf_${wt}_$t.err || { echo "variant $t failed"; tail -5 $OUT/ncf_${wt}_$t.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/ncf_${wt}_$t.out').read().strip().splitlines()[-1]); print('$wt $t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['prefilter']['candidates_per_row'], d['prefilter']['fallback_rows'])"
  done
}
run norms cur cap8 cur cap8
run init cur cap8 cur cap8

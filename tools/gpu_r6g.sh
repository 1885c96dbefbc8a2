set -uo pipefail
OUT=gpurun_out/r6j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "ncf or NCF or prefilter or stress or shard or rccl" --timeout 300 --timeout-method thread > $OUT/tests.out 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.out
run() {  # weights variants...
  local wt=$1; shift
  for t in "$@"; do
    HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 300 python bench.py --workload ncf --weights $wt --profile-only > $OUT/ncf_${wt}_$t.out 2> $OUT/ncf_${wt}_$t.err || { echo "variant $t failed"; tail -5 $OUT/ncf_${wt}_$t.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/ncf_${wt}_$t.out').read().strip().splitlines()[-1]); print('$wt $t', d['value'], d['ms_per_step'], d['roofline'].get('avg_kernel_ms'), d['prefilter']['candidates_per_row'])"
  done
}
run init nbase bf2 nbase bf2 nbase bf2
run personal nbase bf2 nbase bf2
run norms nbase bf2

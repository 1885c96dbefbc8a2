#!/bin/bash
# Whole-step A/B of variant libraries (tools/bin/libhnm_<tag>.so via HNM_LIB_PATH) on one
# bench workload, alternating the variants on the same box.
#   bash tools/gpu_step_ab.sh <workload> "<bench args>" rounds tag1 tag2 ...
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
W=$1; ARGS=$2; N=$3; shift 3
for r in $(seq 1 $N); do
  for t in "$@"; do
    HNM_LIB_PATH=$ROOT/tools/bin/libhnm_$t.so timeout -k 10 300 python $ROOT/bench.py --workload $W $ARGS --no-cpu-baseline --no-extras > /tmp/ab_$t.out 2>/tmp/ab_$t.err || { tail -5 /tmp/ab_$t.err; exit 1; }
    python -c "import json; d=json.loads(open('/tmp/ab_$t.out').read().strip().splitlines()[-1]); print('$t', round(d['value']), d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
  done
done

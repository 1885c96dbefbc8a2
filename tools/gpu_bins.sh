#!/bin/bash
# Run kernel-only timing binaries (tools/bin/<name>) with arguments, alternating, under timeouts.
#   bash tools/gpu_bins.sh <outtag> "<args...>" bin1 bin2 ...   (every binary x every arg, twice)
set -uo pipefail
OUT=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $OUT
for rep in 1 2; do for b in "$@"; do for a in $ARGS; do
  echo -n "$b "; timeout -k 10 60 ./tools/bin/$b $a | tail -1 || exit 1
done; done; done > $OUT/out.txt 2>&1 || { cat $OUT/out.txt; exit 1; }
cat $OUT/out.txt

#!/bin/bash
# SpMM variant sweep: tools/spmm_halves.py (per-half times, sampled forward() rows dumped) per
# variant library at d=64 (and d=128 for the variants after "--"), then a bitwise comparison of
# the dumps against the first variant of each summation-order family.
#   bash tools/gpu_spmm_variants.sh <tag> v1 v2 ... [-- w1 w2 ...]
set -uo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
d=64
for t in "$@"; do
  if [ "$t" = "--" ]; then d=128; continue; fi
  HNM_LIB_PATH=$PWD/tools/bin/libhnm_$t.so timeout -k 10 240 python tools/spmm_halves.py --d $d --reps 10 --dump $OUT/${t}_$d.npz > $OUT/${t}_$d.txt 2> $OUT/${t}_$d.err || { echo "$t d=$d failed"; tail -5 $OUT/${t}_$d.err; exit 1; }
  echo "$t d=$d $(grep -E '^(users|items|layer) ' $OUT/${t}_$d.txt | sed -E "s/'entries'[^,]*,//; s/'gathered_GB'[^,]*,//" | tr '\n' ' ')"
done
echo ok

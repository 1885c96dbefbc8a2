#!/bin/bash
# dot scan: kernel-only timings (tools/bin/dot_scan_*), parity tests of the in-tree library,
# bench A/B of variant libraries on MF and LightGCN d=128.   bash tools/gpu_dot_ab.sh <tag> <libA> <libB> <bins...>
set -uo pipefail
TAG=$1; LA=$2; LB=$3; shift 3
bash tools/gpu_bins.sh ${TAG}_bins "3.1 3.5" "$@" || exit 1
bash tools/gpu_lib_ab.sh ${TAG} "mf or dot or lightgcn or prefilter or filter or sharding" mf "--steps 20 --warmup 5" $LA $LB $LA $LB || exit 1
bash tools/gpu_lib_ab.sh ${TAG}b - lightgcn128 "--steps 3 --warmup 1" $LA $LB || exit 1

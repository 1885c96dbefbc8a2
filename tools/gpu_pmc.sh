#!/bin/bash
# PMC passes (tools/pmc_profile.sh) for several workloads, one after the other.
#   bash tools/gpu_pmc.sh <tag> w1 w2 ...   -> gpurun_out/<tag>_<w>/
set -uo pipefail
TAG=$1; shift
for w in "$@"; do
  echo "== $w $(date +%T)"
  bash tools/pmc_profile.sh $w gpurun_out/${TAG}_$w || exit 1
done
echo ok

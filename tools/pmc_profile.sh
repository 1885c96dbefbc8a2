#!/bin/bash
# rocprofv3 PMC passes for the dominant kernel of a bench workload (run on the GPU box).
# Each counter group is its own pass (kernel-trace only; no sys/runtime trace with --pmc).
#   tools/pmc_profile.sh <workload> <outdir> [extra bench args]
set -euo pipefail
W=${1:-ncf}; OUT=${2:-gpurun_out/pmc}; shift 2 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--workload $W --steps 2 --warmup 1 --profile-only $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/$OUT/p$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$ROOT/$OUT/p$i.log"; exit 1; }
done
echo done

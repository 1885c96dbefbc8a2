#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) over a diagnostic binary.
#   bash tools/pmc_bin.sh <binary> <outdir>
set -euo pipefail
BIN=$1; OUT=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_BRANCH" \
           "SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/$OUT/p$i" -o run -- "$ROOT/$BIN" > "$ROOT/$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$ROOT/$OUT/p$i.log"; exit 1; }
done
echo done

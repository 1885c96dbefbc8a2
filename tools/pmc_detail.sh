#!/bin/bash
# Stall-attribution PMC passes (one counter group per pass, kernel-trace only) for a bench
# workload; summarize with tools/pmc_summary.py-style per-wave means.
#   tools/pmc_detail.sh <workload> <outdir> [extra bench args]
set -euo pipefail
W=${1:-ncf}; OUT=${2:-gpurun_out/pmcd}; shift 2 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--workload $W --steps 2 --warmup 1 --no-cpu-baseline $*"
i=0
for grp in "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_WAVES" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_VMEM SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/$OUT/p$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$ROOT/$OUT/p$i.log"; exit 1; }
done
echo done

#!/bin/bash
# SQ counter passes (stall / instruction mix / LDS conflicts per kernel) over one eager step.
# Usage (GPU box): bash tools/gpu_sq.sh TAG [script.py]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-sq}; PY=${2:-tools/pmc_step.py}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqa" -o run -- python3 "$R/$PY" > "$O/sqa.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqb" -o run -- python3 "$R/$PY" > "$O/sqb.log" 2>&1 && \
python3 "$R/tools/pmc_summary.py" "$O/sqa" "$O/sqb" --top 30 > "$O/summary.txt" 2>&1 && \
python3 "$R/tools/mfma_util.py" "$O/sqb" --top 40 > "$O/mfma_util.txt" 2>&1

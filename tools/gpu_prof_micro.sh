#!/bin/bash
# SQ + traffic counter passes over a micro script: bash tools/gpu_prof_micro.sh TAG script.py
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-micro}; PY=${2:-tools/micro_classattn.py}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqa" -o run -- python3 "$R/$PY" > "$O/sqa.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/sqb" -o run -- python3 "$R/$PY" > "$O/sqb.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/fetch" -o run -- python3 "$R/$PY" > "$O/fetch.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$O/write" -o run -- python3 "$R/$PY" > "$O/write.log" 2>&1 && \
python3 "$R/tools/pmc_summary.py" "$O/sqa" "$O/sqb" "$O/fetch" "$O/write" --top 12 > "$O/summary.txt" 2>&1

#!/bin/bash
# one SQ instruction-mix pass of tools/micro_decoder.py for the library in $1 (CATSEG_HIP_LIB), output dir $2
set -e
O=$2
mkdir -p "$O"
cd /tmp
CATSEG_HIP_LIB=$1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace -f csv -d "$O/sq" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/micro_decoder.py" ring_onebar 1 > "$O/sq.log" 2>&1
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$O/sq" --top 8 > "$O/summary.txt" 2>&1

#!/bin/bash
# Round 4: knob sweeps on the final library (GEMM tile-order group, ring persistence).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04x}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/micro_gemm.py 3004,3000,3002,3006,3008 > $O/micro_gemm_group.log 2>&1 && \
timeout -k 10 200 python -u tools/micro_decoder.py ring_persist 2 1 > $O/micro_decoder_persist.log 2>&1

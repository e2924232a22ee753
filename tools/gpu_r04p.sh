#!/bin/bash
# Round 4 checkpoint after the per-file SLP flags: GPU suite + Swin / class-attention timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04p}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_swin.py 0 > $O/micro_swin.log 2>&1 && \
CA_VARIANTS=0 timeout -k 10 150 python -u tools/micro_classattn.py > $O/micro_classattn.log 2>&1

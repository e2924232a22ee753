#!/bin/bash
# Round 4: ViT attention stagger A/B + attention / hazard tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04e}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/micro_attn.py 0,208,209 > $O/micro_attn.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma_hazard.py tests/test_gpu_ops.py -k "attention or mfma" -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1

#!/bin/bash
# Round 4: software-pipelined ViT attention (attn_variant 1 / 2) tests + A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04n}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention_dense" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_attn.py 200,201,202 > $O/micro_attn.log 2>&1

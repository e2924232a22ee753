#!/bin/bash
# Round 4: merge staging variant + class-attention LayerNorm batch A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04h}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "merge or class_attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_merge.py 2,0,3 > $O/micro_merge.log 2>&1 && \
CA_VARIANTS=0,1,2 timeout -k 10 200 python -u tools/micro_classattn.py > $O/micro_classattn.log 2>&1

#!/bin/bash
# Round 4: one-barrier-per-chunk ring convs (ring_onebar): tests + decoder A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04q}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "ring or upconv" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/micro_decoder.py ring_onebar 0 1 > $O/micro_decoder.log 2>&1

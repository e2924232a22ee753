#!/bin/bash
# GPU iteration: selected op tests ($K over $TESTS), then a same-process A/B of one knob ($KNOB $VALS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py} -m gpu -x -q -k "${K:-.}" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_knob.py $KNOB $VALS > gpurun_out/ab_knob.log 2>&1

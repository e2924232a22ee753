#!/bin/bash
# Quick GPU iteration: selected tests ($K, pytest -k expression over $TESTS) then a bench line without the CPU leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_ops.py}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q -k "${K:-.}" --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --cpu-images 0 > gpurun_out/quick_bench.log 2>&1

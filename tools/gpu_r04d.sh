#!/bin/bash
# Round 4: GPU suite, smoke, headline bench (one call).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04d}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1

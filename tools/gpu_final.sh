#!/bin/bash
# Final check of a build on the GPU box: GPU suite, smoke, headline bench, config-5 bench (no profiling).
# Usage (GPU box): bash tools/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 5 > gpurun_out/$TAG/bench_config5.log 2>&1

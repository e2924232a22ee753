#!/bin/bash
# Quick check of the newest kernels, then the full round-3 evidence (tools/gpu_r03.sh) in one call.
# Usage (GPU box): bash tools/gpu_r03b.sh TAG GIT_HEAD "pytest -k expression" "micro command"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03}; HEAD=${2:-unknown}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "$3" --timeout 120 --timeout-method thread > $O/quick_tests.log 2>&1 || exit 1
if [ -n "$4" ]; then timeout -k 10 240 $4 > $O/quick_micro.log 2>&1 || exit 1; fi
bash tools/gpu_r03.sh $TAG $HEAD

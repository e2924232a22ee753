#!/bin/bash
# Round 4: fp8 GEMM lean prefetching epilogue: tests + config-5 bench + fp8 GEMM micro.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04u}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "gemm" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 5 --cpu-images 0 > $O/bench_config5.log 2>&1

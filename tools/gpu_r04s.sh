#!/bin/bash
# Round 4: gemm3 lean epilogue with the next round's residual in flight (epi_prefetch) test + A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04s}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "gemm" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 200 python -u tools/micro_gemm.py 0,2000 > $O/micro_gemm.log 2>&1 && \
MG_M=2308 timeout -k 10 200 python -u tools/micro_gemm.py 0,2000 > $O/micro_gemm_2308.log 2>&1

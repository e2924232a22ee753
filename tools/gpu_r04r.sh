#!/bin/bash
# Round 4: head-conv prefetch depth / occupancy variants and the postprocess staging, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04r}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "head_conv or postprocess or resize or crops" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_post.py > $O/micro_post_new.log 2>&1 && \
CATSEG_HIP_LIB=$PWD/exp_so/libold_misc.so timeout -k 10 150 python -u tools/micro_post.py 0 > $O/micro_post_old.log 2>&1 && \
timeout -k 10 150 python -u tools/micro_post.py > $O/micro_post_new2.log 2>&1

#!/bin/bash
# Round 4: MLP hidden-tile swizzle A/B, branch-free separable merge, merge SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04g}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "mlp or merge" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_merge.py 2,0,4 > $O/micro_merge.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_mlp.py > $O/micro_mlp_new.log 2>&1 && \
CATSEG_HIP_LIB=$PWD/exp_so/libold_rp.so timeout -k 10 120 python -u tools/micro_mlp.py > $O/micro_mlp_old.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_mlp.py > $O/micro_mlp_new2.log 2>&1 && \
bash tools/gpu_prof_micro.sh $T/merge tools/micro_merge.py

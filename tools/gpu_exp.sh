#!/bin/bash
# Same-box A/B of experiment libraries (tools/build_exp.sh): runs CMD once with the default library,
# then once per exp_so/lib<NAME>.so, then the default again.
# Usage: CMD="python tools/micro_swin.py 0" bash tools/gpu_exp.sh TAG NAME1 NAME2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 150 $CMD > $O/base.log 2>&1 || exit 1
for n in "$@"; do
  CATSEG_HIP_LIB=$PWD/exp_so/lib$n.so timeout -k 10 150 $CMD > $O/$n.log 2>&1 || exit 1
done
timeout -k 10 150 $CMD > $O/base2.log 2>&1

#!/bin/bash
# One iteration on the GPU box: selected GPU tests ($K over $TESTS), then the commands in $MICRO
# (";"-separated, each under its own limit), then a headline bench line without the CPU leg.
# Usage: K=expr TESTS="tests/x.py" MICRO="python tools/a.py 1 0;python tools/b.py" bash tools/gpu_iter.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-iter}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py} -m gpu -x -q -k "${K:-.}" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
i=0
IFS=';' read -ra CMDS <<< "$MICRO"
for c in "${CMDS[@]}"; do
  [ -z "$c" ] && continue
  i=$((i+1))
  timeout -k 10 240 $c > $O/micro$i.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --cpu-images 0 > $O/bench.log 2>&1

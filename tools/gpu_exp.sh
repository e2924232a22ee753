#!/bin/bash
# Experiment call: each argument is one python command line (run from the repo root) under its own
# time limit, output to gpurun_out/exp_<i>.log; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cmd in "$@"; do
  i=$((i + 1))
  echo "== $cmd" > gpurun_out/exp_$i.log
  timeout -k 10 ${EXP_TIMEOUT:-300} python -u $cmd >> gpurun_out/exp_$i.log 2>&1 || { rc=$?; echo "step $i failed rc=$rc"; tail -5 gpurun_out/exp_$i.log; exit $rc; }
  cat gpurun_out/exp_$i.log
done

#!/bin/bash
# Round 4 final check of a build: GPU suite, smoke, headline + configs 2 / 4 / 5 bench lines, the MFMA
# overlap probe.  Usage (GPU box): bash tools/gpu_r04_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04f}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
bash tools/gpu_r04_bench.sh $T

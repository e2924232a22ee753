#!/bin/bash
# Round 4 profiler evidence for the current build: rocprofv3 kernel-trace stats of the bench command,
# FETCH_SIZE / WRITE_SIZE PMC passes, SQ passes.  Usage (GPU box): bash tools/gpu_r04_evidence.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04e}
mkdir -p gpurun_out/$T
bash tools/gpu_evidence.sh $T

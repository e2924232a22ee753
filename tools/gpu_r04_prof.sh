#!/bin/bash
# Round 4 evidence for the current build: headline bench line, rocprofv3 kernel trace, FETCH / WRITE
# PMC passes, SQ passes (tools/gpu_profile.sh + tools/gpu_sq.sh).  Usage: bash tools/gpu_r04_prof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04p}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/$T/bench.log 2>&1 && \
bash tools/gpu_evidence.sh $T

#!/bin/bash
# rocprofv3 evidence: kernel-trace stats + FETCH/WRITE traffic passes + SQ passes. Usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-r02}
bash "$R/tools/gpu_profile.sh" "$TAG" && bash "$R/tools/gpu_sq.sh" "$TAG/sq"

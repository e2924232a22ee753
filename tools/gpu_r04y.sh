#!/bin/bash
# Round 4 final library: GPU suite + smoke + bench lines (tools/gpu_r04_final.sh), then knob sweeps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04v4}
bash tools/gpu_r04_final.sh $T && bash tools/gpu_r04x.sh $T/sweep

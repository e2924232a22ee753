#!/bin/bash
# Config-5 evidence (sliding 640², pc459, fp8 ViT GEMMs): bench line + rocprofv3 kernel stats.
# Usage (GPU box): bash tools/gpu_config5.sh TAG
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-c5}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 400 python3 "$R/bench.py" --config 5 --steps 5 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/bench.py" --config 5 --steps 3 --warmup 1 --cpu-images 0 --no-roofline > "$O/trace.log" 2>&1

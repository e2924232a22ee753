#!/bin/bash
# A/B two library builds on one box: bench + kernel-trace stats for each.
# Usage: bash tools/_ab.sh ALT_SO_PATH
set -o pipefail
R="$GRAFT_REPO_ROOT"; ALT="$1"; O="$R/gpurun_out/ab"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-images 0 > "$O/bench_a.json" 2> "$O/a.err" && \
CATSEG_HIP_LIB="$ALT" timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-images 0 > "$O/bench_b.json" 2> "$O/b.err" && \
timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-images 0 > "$O/bench_a2.json" 2>> "$O/a.err" && \
CATSEG_HIP_LIB="$ALT" timeout -k 10 200 python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-images 0 > "$O/bench_b2.json" 2>> "$O/b.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/ta" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-images 0 > "$O/ta.log" 2>&1 && \
CATSEG_HIP_LIB="$ALT" timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/tb" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-images 0 > "$O/tb.log" 2>&1

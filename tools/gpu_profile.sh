#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench command, then one
# FETCH_SIZE and one WRITE_SIZE PMC pass (each its own run) over tools/pmc_step.py.
# Usage (GPU box): bash tools/gpu_profile.sh TAG [GIT_HEAD]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${1:-r01}; HEAD=${2:-unknown}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-images 0 > "$O/trace.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$O/pmc_fetch" -o run -- python3 "$R/tools/pmc_step.py" > "$O/pmc_fetch.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$O/pmc_write" -o run -- python3 "$R/tools/pmc_step.py" > "$O/pmc_write.log" 2>&1 && \
python3 "$R/tools/pmc_traffic.py" "$O/pmc_fetch" "$O/pmc_write" -o "$O/pmc_traffic.json" --head "$HEAD" > "$O/pmc_traffic.txt" 2>&1

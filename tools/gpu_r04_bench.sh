#!/bin/bash
# Round 4 bench lines for the current build: smoke, headline, configs 2 / 4 / 5, the MFMA overlap probe.
# Usage (GPU box): bash tools/gpu_r04_bench.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config 2 > $O/bench_config2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_config4.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 5 > $O/bench_config5.log 2>&1 && \
timeout -k 10 120 ./tools/bin/probe_mfma_overlap 32 > $O/probe_mfma_overlap.txt 2>&1

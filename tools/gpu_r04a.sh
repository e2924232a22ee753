#!/bin/bash
# Round 4, first call: MFMA operand-overlap probe, the GPU suite, smoke, headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04a}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/probe_mfma_overlap.hip -o /tmp/probe_mfma_overlap > gpurun_out/$TAG/probe_build.log 2>&1 && \
timeout -k 10 120 /tmp/probe_mfma_overlap > gpurun_out/$TAG/probe.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1

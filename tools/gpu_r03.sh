#!/bin/bash
# Round-3 evidence in one call (GPU box): GPU suite, smoke, headline bench, config 2/4/5 bench lines,
# then rocprofv3 kernel-trace stats + FETCH/WRITE PMC passes (lib sha + git head recorded) + SQ passes
# with MFMA busy per kernel.  Usage: bash tools/gpu_r03.sh TAG GIT_HEAD [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03}; HEAD=${2:-unknown}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config 2 > $O/bench_config2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config 4 > $O/bench_config4.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 5 --cpu-images 0 > $O/bench_config5.log 2>&1 && \
bash tools/gpu_profile.sh $TAG $HEAD && bash tools/gpu_sq.sh $TAG/sq

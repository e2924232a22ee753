#!/bin/bash
# Round-2 GPU call: focused tests ($FOCUS), full GPU suite, smoke, bench (each step time-limited, chained with &&).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
FOCUS=${FOCUS:-tests/test_gpu_parity_bench.py}
timeout -k 10 700 python -u -m pytest $FOCUS -m gpu -v -s --timeout 900 --timeout-method thread > gpurun_out/focus.log 2>&1
rc=$?
echo "focus rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ -n "$SKIP_SUITE" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --ignore tests/test_gpu_parity_bench.py --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1

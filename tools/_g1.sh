set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity_bench.py tests/test_gpu_e2e.py -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1

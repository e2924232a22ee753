set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundary.py -x -v --timeout 300 --timeout-method thread > $O/tests_boundary.log 2>&1 &&
timeout -k 10 400 python -u bench.py --cpu-images 0 > $O/bench1.json 2> $O/bench1.err &&
timeout -k 10 400 python -u tools/probe_boundary.py > $O/probe_boundary.log 2>&1

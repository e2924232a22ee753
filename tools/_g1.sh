cd $GRAFT_REPO_ROOT && O=gpurun_out/r06l && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_boundary.py -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1

cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06t &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_ops.py -k "vpt or full" -x -v --timeout 300 --timeout-method thread > gpurun_out/r06t/tests.log 2>&1

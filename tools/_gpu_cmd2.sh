R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -x -v -s --timeout 300 --timeout-method thread -k "l14" > gpurun_out/t.log 2>&1

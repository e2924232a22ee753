cd $GRAFT_REPO_ROOT && O=gpurun_out/r06m && mkdir -p $O &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e.py -k "l14_options" -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1

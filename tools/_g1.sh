# scratch launcher for one-off gpurun calls (the maintained launcher is tools/gpu.sh)
cd $GRAFT_REPO_ROOT && O=gpurun_out/scratch && mkdir -p $O &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1

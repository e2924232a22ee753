R="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "corr_embed or class_attention" > gpurun_out/t.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --cpu-images 0 --steps 20 > gpurun_out/bench.log 2>&1

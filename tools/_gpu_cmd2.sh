R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python -u tools/micro_gemm.py > gpurun_out/micro_gemm.log 2>&1 && \
timeout -k 10 200 python -u bench.py --cpu-images 0 --steps 20 > gpurun_out/bench.log 2>&1

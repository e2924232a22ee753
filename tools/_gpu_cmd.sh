timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread -k "gemm or swin or golden or config2" > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python -u bench.py --cpu-images 0 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 120 python -u tools/micro_gemm.py 5,9 > gpurun_out/micro_gemm.log 2>&1

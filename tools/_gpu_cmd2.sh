R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python -u bench.py --cpu-images 0 --steps 20 > gpurun_out/bench.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/kt" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-images 0 --no-roofline > "$R/gpurun_out/kt.log" 2>&1

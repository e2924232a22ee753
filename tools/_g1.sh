cd $GRAFT_REPO_ROOT && O=gpurun_out/r06v && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread > $O/tests_bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --config 2 --cpu-images 0 > $O/bench_config2.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --config 4 --cpu-images 0 > $O/bench_config4.json 2>> $O/bench.err &&
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-images 0 > $O/bench_config5.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --cpu-images 0 --attention-type full > $O/bench_full_attention.json 2>> $O/bench.err &&
timeout -k 10 300 python -u bench.py --cpu-images 0 --prompt-length 10 > $O/bench_vpt10.json 2>> $O/bench.err

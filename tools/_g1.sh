cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06u &&
timeout -k 10 300 python -u bench.py --cpu-images 0 --no-boundary > gpurun_out/r06u/bench.json 2> gpurun_out/r06u/bench.err &&
timeout -k 10 300 python -u bench.py --config 4 --cpu-images 0 > gpurun_out/r06u/bench_config4.json 2>> gpurun_out/r06u/bench.err

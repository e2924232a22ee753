cd $GRAFT_REPO_ROOT && O=gpurun_out/r06i && mkdir -p $O &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --config 4 --cpu-images 0 > $O/bench_config4.json 2>> $O/bench.err

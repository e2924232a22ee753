cd $GRAFT_REPO_ROOT && O=gpurun_out/r06h && mkdir -p $O &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err

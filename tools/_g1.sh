cd $GRAFT_REPO_ROOT && O=gpurun_out/r06x && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_e2e.py -k "full" -x -v --timeout 300 --timeout-method thread > $O/tests_full.log 2>&1 &&
timeout -k 10 200 env CATSEG_HIP_LIB=$GRAFT_REPO_ROOT/exp_so/libold.so python -u bench.py --cpu-images 0 --attention-type full > $O/old_full.json 2>> $O/bench.err &&
timeout -k 10 200 python -u bench.py --cpu-images 0 --attention-type full > $O/new_full.json 2>> $O/bench.err &&
timeout -k 10 200 env CATSEG_HIP_LIB=$GRAFT_REPO_ROOT/exp_so/libold.so python -u bench.py --cpu-images 0 --attention-type full > $O/old_full2.json 2>> $O/bench.err &&
timeout -k 10 200 python -u bench.py --cpu-images 0 --attention-type full > $O/new_full2.json 2>> $O/bench.err

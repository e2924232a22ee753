cd $GRAFT_REPO_ROOT && O=gpurun_out/r06w && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3 or conv or guidance" -x -q --timeout 300 --timeout-method thread > $O/tests_conv.log 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 200 env CATSEG_HIP_LIB=$GRAFT_REPO_ROOT/exp_so/libold.so python -u bench.py --cpu-images 0 --no-boundary > $O/old_$i.json 2>> $O/bench.err &&
  timeout -k 10 200 python -u bench.py --cpu-images 0 --no-boundary > $O/new_$i.json 2>> $O/bench.err || exit 1
done &&
timeout -k 10 200 env CATSEG_HIP_LIB=$GRAFT_REPO_ROOT/exp_so/libold.so python -u bench.py --config 2 --cpu-images 0 > $O/old_c2.json 2>> $O/bench.err &&
timeout -k 10 200 python -u bench.py --config 2 --cpu-images 0 > $O/new_c2.json 2>> $O/bench.err

cd $GRAFT_REPO_ROOT && O=gpurun_out/r06n && mkdir -p $O &&
for i in 1 2 3; do
  timeout -k 10 200 env CATSEG_BENCH_GRAPHS=1 python -u bench.py --cpu-images 0 --no-boundary --no-roofline --steps 20 > $O/g1_$i.json 2>> $O/bench.err &&
  timeout -k 10 200 env CATSEG_BENCH_GRAPHS=2 python -u bench.py --cpu-images 0 --no-boundary --no-roofline --steps 20 > $O/g2_$i.json 2>> $O/bench.err || exit 1
done

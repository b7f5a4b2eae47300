set -e
cd $GRAFT_REPO_ROOT
for P in 90 120; do
  timeout -k 10 500 python bench.py --steps 8 --warmup 1 --pairs-per-step $P > gpurun_out/bench_tuned_P$P.log 2>&1 || true
  echo "P=$P"; tail -1 gpurun_out/bench_tuned_P$P.log | cut -c1-160
done

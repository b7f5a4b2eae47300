set -e
cd $GRAFT_REPO_ROOT
for P in 4 8 15; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --pairs-per-step $P --profile-steps > gpurun_out/bs_P$P.log 2>&1
  tail -1 gpurun_out/bs_P$P.log | cut -c1-200
done
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --pairs-per-step 15 --no-nll > gpurun_out/bs_P15_nonll.log 2>&1
tail -1 gpurun_out/bs_P15_nonll.log | cut -c1-200

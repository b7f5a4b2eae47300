set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
echo SMOKE_OK
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --profile-steps > gpurun_out/bench1.log 2>&1
echo BENCH_OK

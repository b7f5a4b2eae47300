set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-tuned-gemms > gpurun_out/ab_untuned.log 2>&1
tail -1 gpurun_out/ab_untuned.log | cut -c1-150
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_tuned.log 2>&1
tail -1 gpurun_out/ab_tuned.log | cut -c1-150

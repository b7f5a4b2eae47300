set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kt2.log 2>&1; tail -1 gpurun_out/kt2.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --profile-steps > gpurun_out/ab_share.log 2>&1
tail -1 gpurun_out/ab_share.log | cut -c1-220
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-prefix-share > gpurun_out/ab_noshare.log 2>&1
tail -1 gpurun_out/ab_noshare.log | cut -c1-220

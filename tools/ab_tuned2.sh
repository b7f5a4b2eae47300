set -e
cd $GRAFT_REPO_ROOT
TB_PHASE_TIMING=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/ab2_tuned.log 2>&1
grep step gpurun_out/ab2_tuned.log; tail -1 gpurun_out/ab2_tuned.log | cut -c1-150
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-tuned-gemms > gpurun_out/ab2_untuned.log 2>&1
tail -1 gpurun_out/ab2_untuned.log | cut -c1-150
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/ab2_tuned_nt.log 2>&1
tail -1 gpurun_out/ab2_tuned_nt.log | cut -c1-150

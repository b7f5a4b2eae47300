set -e
cd $GRAFT_REPO_ROOT
for P in 30 45; do
TB_PHASE_TIMING=1 timeout -k 10 500 python bench.py --steps 2 --warmup 1 --pairs-per-step $P --profile-steps --no-tuned-gemms > gpurun_out/bs2_P$P.log 2>&1
grep "step 2" gpurun_out/bs2_P$P.log | cut -c1-220; tail -1 gpurun_out/bs2_P$P.log | cut -c1-150
done

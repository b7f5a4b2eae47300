#!/bin/bash
# Driver-shaped bench (20 timed steps, 5 warmup) on HEAD, then the 9B projection sweep with gradient
# directions (EP:146 alternative) vs PCA.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/long
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/long/bench_20_5.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/long/bench_20_5.log
for sub in pca grad_model grad_lens; do
timeout -k 10 600 python -m taboo_brittleness_amd run_sweep configs/ll_baseline_9b.yaml --methods proj --set intervention.subspace=$sub --set runtime.batch_size=4096 --out gpurun_out/long/sweep_$sub > gpurun_out/long/sweep_$sub.log 2>&1
echo SWEEP_$sub; tail -1 gpurun_out/long/sweep_$sub.log
done

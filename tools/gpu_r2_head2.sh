#!/bin/bash
# Fused vocab head in the engine: full GPU tier, then bench with and without it (same box, alternating).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/head2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/head2/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/head2/pytest_gpu.log
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/head2/bench_fused_$i.log 2>&1
echo FUSED_$i; tail -1 gpurun_out/head2/bench_fused_$i.log | cut -c1-200
timeout -k 10 400 python bench.py --no-fused-head > gpurun_out/head2/bench_unfused_$i.log 2>&1
echo UNFUSED_$i; tail -1 gpurun_out/head2/bench_unfused_$i.log | cut -c1-200
done

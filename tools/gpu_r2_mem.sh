#!/bin/bash
# Lazy running lens sums: GPU tier, default bench, then the bench at 110 / 120 pairs per step (memory headroom).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -1 gpurun_out/pytest_gpu.log
for P in 90 120; do
  timeout -k 10 600 python bench.py --steps 8 --warmup 1 --pairs-per-step $P > gpurun_out/bench_P$P.log 2>&1 || true
  echo "P=$P"; tail -1 gpurun_out/bench_P$P.log | cut -c1-200; grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/bench_P$P.log || true
done

#!/bin/bash
# Tail vocab-head rows per fused-head GEMM: whole chunks (16384) vs 2048, same box, alternating.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/headrows
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/headrows/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/headrows/pytest_gpu.log
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/headrows/bench_16384_$i.log 2>&1
echo R16384_$i; tail -1 gpurun_out/headrows/bench_16384_$i.log | cut -c1-130
TB_TF_HEAD_ROWS=2048 timeout -k 10 400 python bench.py > gpurun_out/headrows/bench_2048_$i.log 2>&1
echo R2048_$i; tail -1 gpurun_out/headrows/bench_2048_$i.log | cut -c1-130
done

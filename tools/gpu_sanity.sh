#!/bin/bash
# Round sanity pass on one MI355X: GPU test tier, smoke, default bench.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
echo SMOKE_OK; tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/bench_default.log

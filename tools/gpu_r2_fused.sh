#!/bin/bash
# GEMM-kernel tests, then the default bench and the fused-GeGLU bench back to back on one box.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/pytest_gemm.log 2>&1
echo TESTS_OK; tail -1 gpurun_out/pytest_gemm.log
timeout -k 10 400 python bench.py > gpurun_out/bench_unfused.log 2>&1
echo UNFUSED; tail -1 gpurun_out/bench_unfused.log
timeout -k 10 400 python bench.py --fused-geglu > gpurun_out/bench_fused.log 2>&1
echo FUSED; tail -1 gpurun_out/bench_fused.log

#!/bin/bash
# Fused vocab head: GPU numerics test, then the A/B microbenchmark at Gemma-2-9B shapes.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/head
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "vocab_head or decode_head or gemm_pp" > gpurun_out/head/pytest.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/head/pytest.log
timeout -k 10 300 python tools/head_bench.py > gpurun_out/head/head_bench.log 2>&1
echo BENCH_OK; cat gpurun_out/head/head_bench.log

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" \
  > gpurun_out/r6/pytest_attn.log 2>&1 || exit 2
TB_EXACT_OUT=gpurun_out/r6 timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_exact_9b_gpu.py tests/test_bench_gpu.py > gpurun_out/r6/pytest_9b.log 2>&1 || exit 3

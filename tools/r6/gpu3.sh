#!/bin/bash
# round 6: the 9B exactness and 2-rank bench tests, LoRA GPU tests, GEMM kernel tests
set -o pipefail
mkdir -p gpurun_out/r6
TB_EXACT_OUT=gpurun_out/r6 timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_exact_9b_gpu.py tests/test_bench_gpu.py > gpurun_out/r6/pytest_9b.log 2>&1; r1=$?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_lora_gpu.py \
  > gpurun_out/r6/pytest_lora.log 2>&1; r2=$?
[ $r2 -le 1 ] || exit 2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or ring or attention" \
  > gpurun_out/r6/pytest_kern.log 2>&1 || exit 3
exit $(( r1 + r2 ))

#!/bin/bash
# round 6: the 9B exactness and 2-rank bench tests
set -o pipefail
mkdir -p gpurun_out/r6
TB_EXACT_OUT=gpurun_out/r6 timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_exact_9b_gpu.py tests/test_bench_gpu.py > gpurun_out/r6/pytest_9b.log 2>&1 || exit 3

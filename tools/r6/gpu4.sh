#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u tools/r6/debug_exact.py > gpurun_out/r6/debug_exact.log 2>&1; r1=$?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_lora_gpu.py \
  > gpurun_out/r6/pytest_lora.log 2>&1; r2=$?
exit $(( r1 + r2 ))

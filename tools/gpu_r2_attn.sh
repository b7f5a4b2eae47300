#!/bin/bash
# Decode-attention kernel A/B: GPU tests on the new kernel, attn_scan legacy vs one-wave-per-head.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
echo TESTS_OK; tail -1 gpurun_out/pytest_attn.log
TB_ATTN_DECODE_LEGACY=1 timeout -k 10 120 python tools/attn_scan.py > gpurun_out/attn_scan_legacy.log 2>&1
timeout -k 10 120 python tools/attn_scan.py > gpurun_out/attn_scan_wave.log 2>&1
echo SCAN_OK

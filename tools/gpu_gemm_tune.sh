#!/bin/bash
# GEMM kernel tests (tile variants, batch invariance) then the dispatch-table measurement.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/gemm
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm or linear" > gpurun_out/gemm/pytest.log 2>&1
echo TESTS_OK; tail -2 gpurun_out/gemm/pytest.log
timeout -k 10 900 python -u tools/gemm_dispatch_tune.py --raw gpurun_out/gemm/raw.jsonl --out gpurun_out/gemm/gemma2-9b.json "$@" > gpurun_out/gemm/tune.log 2>&1
echo TUNE_OK; tail -2 gpurun_out/gemm/tune.log

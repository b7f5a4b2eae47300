#!/bin/bash
# Cascade decode-attention: kernel tests, full GPU tier, then bench A/B (cascade on / off) on one box.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
echo ATTN_OK; tail -1 gpurun_out/pytest_attn.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 8 --warmup 1 > gpurun_out/bench_casc.log 2>&1
echo BENCH_CASC; tail -1 gpurun_out/bench_casc.log | cut -c1-200
TB_ATTN_CASCADE=0 timeout -k 10 600 python bench.py --steps 8 --warmup 1 > gpurun_out/bench_nocasc.log 2>&1
echo BENCH_NOCASC; tail -1 gpurun_out/bench_nocasc.log | cut -c1-200

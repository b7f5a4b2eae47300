#!/bin/bash
# Decode-attention variants: kernel tests, GPU tier, kernel stats A/B (cascade off / on).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -1 gpurun_out/pytest_gpu.log
bash tools/prof_ab_stats.sh attn TB_ATTN_CASCADE=0 TB_ATTN_CASCADE=1 --steps 2 --warmup 1

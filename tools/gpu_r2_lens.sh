#!/bin/bash
# Fused lens unembed + XCD-remapped decode attention: GPU tier, then bench A/B (same box, alternating).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/lens
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/lens/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/lens/pytest_gpu.log
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/lens/bench_default_$i.log 2>&1
echo DEFAULT_$i; tail -1 gpurun_out/lens/bench_default_$i.log | cut -c1-130
TB_FUSED_LENS=0 timeout -k 10 400 python bench.py > gpurun_out/lens/bench_nolens_$i.log 2>&1
echo NOLENS_$i; tail -1 gpurun_out/lens/bench_nolens_$i.log | cut -c1-130
TB_ATTN_XCD=1 timeout -k 10 400 python bench.py > gpurun_out/lens/bench_xcd_$i.log 2>&1
echo XCD_$i; tail -1 gpurun_out/lens/bench_xcd_$i.log | cut -c1-130
done

#!/bin/bash
# Bench A/B of the decode-attention kernels (same box, back to back).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TB_ATTN_DECODE_LEGACY=1 timeout -k 10 400 python bench.py > gpurun_out/bench_attn_legacy.log 2>&1
echo LEGACY; tail -1 gpurun_out/bench_attn_legacy.log | cut -c1-160
timeout -k 10 400 python bench.py > gpurun_out/bench_attn_wave.log 2>&1
echo WAVE; tail -1 gpurun_out/bench_attn_wave.log | cut -c1-160
timeout -k 10 400 python bench.py --fused-geglu > gpurun_out/bench_attn_wave_fused.log 2>&1
echo WAVE_FUSED; tail -1 gpurun_out/bench_attn_wave_fused.log | cut -c1-160

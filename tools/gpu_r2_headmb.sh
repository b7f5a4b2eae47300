#!/bin/bash
# Tail vocab-head chunk size with the hipBLASLt head (TB_TF_HEAD_MB: MB of bf16 logits per GEMM), one box.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/headmb
for mb in 1024 2048 4096 1024; do
  timeout -k 10 500 env TB_TF_HEAD_MB=$mb python bench.py --steps 8 --warmup 2 > gpurun_out/headmb/bench_$mb.log 2>&1
  echo "MB=$mb"; tail -1 gpurun_out/headmb/bench_$mb.log | cut -c60-100
done

#!/bin/bash
# Extend the P90 TunableOp table with the prefix-trie decode's GEMM shapes, bench with it, kernel-stats profile.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop gpurun_out/trie
cp configs/tunableop/gemma2-9b_P90_E4_new50.csv gpurun_out/tunableop/gemma2-9b_P90_E4_new50.csv
timeout -k 10 1000 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/trie/tune_p90.log 2>&1
echo TUNE_OK; tail -1 gpurun_out/trie/tune_p90.log | cut -c1-200; wc -l gpurun_out/tunableop/*.csv
timeout -k 10 600 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop python bench.py --steps 8 --warmup 1 > gpurun_out/trie/bench_tuned8.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/trie/bench_tuned8.log

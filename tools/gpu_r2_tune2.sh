#!/bin/bash
# Extend the P90 TunableOp table with the end-of-round-2 GEMM shapes (trie decode lo rows, no-op-skip tail chunks,
# padded dedup lens chunks), then A/B the bench with the extended table vs the committed one (one box).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune2/tab
cp configs/tunableop/gemma2-9b_P90_E4_new50.csv gpurun_out/tune2/tab/
timeout -k 10 900 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tune2/tab python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/tune2/tune.log 2>&1
echo TUNE_OK; wc -l gpurun_out/tune2/tab/*.csv
timeout -k 10 500 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tune2/tab python bench.py --steps 8 --warmup 2 > gpurun_out/tune2/bench_new.log 2>&1
echo NEW; tail -1 gpurun_out/tune2/bench_new.log | cut -c60-100
timeout -k 10 500 python bench.py --steps 8 --warmup 2 > gpurun_out/tune2/bench_old.log 2>&1
echo OLD; tail -1 gpurun_out/tune2/bench_old.log | cut -c60-100

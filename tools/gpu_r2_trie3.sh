#!/bin/bash
# Prefix-trie decode + lens row dedup: GPU tests, TunableOp extension for the new shapes, bench with it.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop gpurun_out/trie
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fanout or trie or rowmap or readouts or layer_resume or carry or pipeline" > gpurun_out/trie/pytest3.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/trie/pytest3.log
timeout -k 10 400 python bench.py > gpurun_out/trie/bench_dedup.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/trie/bench_dedup.log
cp configs/tunableop/gemma2-9b_P90_E4_new50.csv gpurun_out/tunableop/gemma2-9b_P90_E4_new50.csv
timeout -k 10 1000 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/trie/tune_p90.log 2>&1
echo TUNE_OK; wc -l gpurun_out/tunableop/*.csv
timeout -k 10 600 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop python bench.py --steps 8 --warmup 1 > gpurun_out/trie/bench_tuned8.log 2>&1
echo BENCH_TUNED; tail -1 gpurun_out/trie/bench_tuned8.log

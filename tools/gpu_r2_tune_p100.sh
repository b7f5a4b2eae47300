#!/bin/bash
# Extend the P100 TunableOp table (seeded from P90) with the P100 bench's shapes, then the driver-shaped bench.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune_p100/tab
cp configs/tunableop/gemma2-9b_P100_E4_new50.csv gpurun_out/tune_p100/tab/
timeout -k 10 900 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tune_p100/tab python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/tune_p100/tune.log 2>&1
echo TUNE_OK; wc -l gpurun_out/tune_p100/tab/*.csv
timeout -k 10 800 env TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tune_p100/tab python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/tune_p100/bench_20_5.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/tune_p100/bench_20_5.log | cut -c1-200

#!/bin/bash
# TunableOp over the GEMM shapes of the default bench not yet in configs/tunableop (init gain 32,
# row-bucketed decode), then an A/B of tuned vs untuned.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop
cp configs/tunableop/gemma2-9b_P60_E4_new50.csv gpurun_out/tunableop/gemma2-9b_P90_E4_new50.csv
export TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop
timeout -k 10 800 python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/tune_g32.log 2>&1 || echo "tuning pass ended rc=$?"
wc -l gpurun_out/tunableop/*.csv
timeout -k 10 300 python bench.py > gpurun_out/bench_tuned.log 2>&1
tail -1 gpurun_out/bench_tuned.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tuned', d['value'], d['ms_per_step'], d['work'])"
timeout -k 10 300 python bench.py --no-tuned-gemms > gpurun_out/bench_untuned.log 2>&1
tail -1 gpurun_out/bench_untuned.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('untuned', d['value'], d['ms_per_step'])"

#!/bin/bash
# TunableOp over every GEMM shape of the P=60 bench, then an A/B of tuned vs untuned.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop
export TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop
timeout -k 10 800 python bench.py --steps 1 --warmup 1 --tune-gemms > gpurun_out/tune_p60.log 2>&1
tail -1 gpurun_out/tune_p60.log | cut -c1-120
ls -la gpurun_out/tunableop
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_tuned.log 2>&1
tail -1 gpurun_out/bench_tuned.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tuned', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-tuned-gemms > gpurun_out/bench_untuned.log 2>&1
tail -1 gpurun_out/bench_untuned.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('untuned', d['value'], d['ms_per_step'])"

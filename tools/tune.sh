#!/bin/bash
# TunableOp over every GEMM shape of the default bench, then tuned vs untuned A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop
export TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop
timeout -k 10 900 python bench.py --tune-gemms "$@" > gpurun_out/tune.log 2>&1
tail -1 gpurun_out/tune.log | cut -c1-120
ls gpurun_out/tunableop
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_tuned.log 2>&1
tail -1 gpurun_out/bench_tuned.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tuned', d['value'], d['ms_per_step'])"
timeout -k 10 400 python bench.py --no-tuned-gemms "$@" > gpurun_out/bench_untuned.log 2>&1
tail -1 gpurun_out/bench_untuned.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('untuned', d['value'], d['ms_per_step'])"

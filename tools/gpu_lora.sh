#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for R in 8 0; do
  timeout -k 10 500 python bench.py --steps 3 --warmup 1 --lora-rank $R > gpurun_out/bench_lora$R.log 2>&1
  tail -1 gpurun_out/bench_lora$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lora=$R', d['value'], d['ms_per_step'], d['work'])"
done

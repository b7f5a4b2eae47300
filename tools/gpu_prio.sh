#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for PR in -1 0; do
  TB_SIDE_PRIORITY=$PR timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_pr$PR.log 2>&1
  tail -1 gpurun_out/bench_pr$PR.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prio=$PR', d['value'], d['ms_per_step'])"
done

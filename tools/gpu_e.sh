#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for E in 4 2 1; do
  timeout -k 10 600 python bench.py --steps 4 --warmup 1 --baseline-every $E > gpurun_out/bench_E$E.log 2>&1
  tail -1 gpurun_out/bench_E$E.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('E=$E', d['value'], d['ms_per_step'], d['config']['baseline_every'])"
done

#!/bin/bash
# Phase-timed bench at several pairs-per-step values: tools/bench_p.sh 30 60 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for P in "$@"; do
  TB_PHASE_TIMING=1 timeout -k 10 500 python bench.py --steps 3 --warmup 1 --pairs-per-step $P --profile-steps > gpurun_out/bench_P$P.log 2>&1
  grep "step 3" gpurun_out/bench_P$P.log | cut -c1-400
  tail -1 gpurun_out/bench_P$P.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('P=$P', d['value'], d['ms_per_step'], d['work'])"
done

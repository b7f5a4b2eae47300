#!/bin/bash
# GPU tests, then the flagship bench (no phase syncs) with and without the ride-along overlap.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for OV in 1 0; do
  TB_OVERLAP_RIDE=$OV timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_ov$OV.log 2>&1
  tail -1 gpurun_out/bench_ov$OV.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap=$OV', d['value'], d['ms_per_step'], d['work'])"
done

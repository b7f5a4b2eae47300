#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/gpu_kt.log 2>&1 || { tail -40 gpurun_out/gpu_kt.log; exit 1; }
tail -1 gpurun_out/gpu_kt.log
for SK in 64 0; do
  TB_SKINNY_MAX_M=$SK timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_sk$SK.log 2>&1
  tail -1 gpurun_out/bench_sk$SK.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('skinny<=$SK', d['value'], d['ms_per_step'])"
done
TB_OVERLAP_RIDE=0 TB_PHASE_TIMING=1 timeout -k 10 500 python bench.py --steps 2 --warmup 1 --profile-steps > gpurun_out/bench_sk_phases.log 2>&1
grep "step 2" gpurun_out/bench_sk_phases.log | cut -c1-400

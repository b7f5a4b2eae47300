#!/bin/bash
# One GPU iteration: kernel + engine tests, then the flagship bench with per-phase timing.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TB_PHASE_TIMING=1 timeout -k 10 500 python bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench_iter.log 2>&1
grep -i "step\|phase" gpurun_out/bench_iter.log | cut -c1-300 | tail -8; tail -1 gpurun_out/bench_iter.log | cut -c1-250

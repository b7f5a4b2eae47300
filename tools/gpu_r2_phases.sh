#!/bin/bash
# GPU tier + per-phase wall times of the default bench (phases synchronised: TB_PHASE_TIMING=1).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/pytest_gpu.log
TB_PHASE_TIMING=1 timeout -k 10 600 python bench.py --steps 4 --warmup 1 --profile-steps > gpurun_out/bench_phases.log 2>&1
echo PHASES_OK; tail -6 gpurun_out/bench_phases.log | cut -c1-900

#!/bin/bash
# Default bench (init gain 32), per-phase timings, and a rocprofv3 kernel-stats pass.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --profile-steps > gpurun_out/b_g32.log 2>&1
echo B_OK; tail -1 gpurun_out/b_g32.log
TB_PHASE_TIMING=1 timeout -k 10 400 python bench.py --steps 2 --profile-steps > gpurun_out/b_g32_phase.log 2>&1
echo PH_OK; grep "step" gpurun_out/b_g32_phase.log | cut -c1-900
bash tools/prof_stats.sh g32 --steps 2

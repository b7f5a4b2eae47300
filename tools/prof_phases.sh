#!/bin/bash
# Kernel trace + per-phase attribution of the default bench (phases synchronised, TB_PHASE_TIMING=1).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_TIMING=1 TB_PHASE_MARKS=$R/gpurun_out/phase_marks.json
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_ph -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_ph.log 2>&1
echo PROF_OK
tail -1 $R/gpurun_out/prof_ph.log | cut -c1-150

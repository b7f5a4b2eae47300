#!/bin/bash
# Kernel-level profile of the flagship bench: rocprofv3 --kernel-trace --stats (no PMC counters).
# Usage: tools/prof_stats.sh <tag> [bench args...]
set -e
TAG=${1:-run}; shift || true
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
echo PROF_OK
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-200
find $R/gpurun_out/prof_$TAG -name "*kernel_stats*" -exec head -25 {} \; | cut -c1-150
# the per-dispatch trace is hundreds of MB: keep the stats only (gpurun copies back <= 64 MiB)
find $R/gpurun_out/prof_$TAG -name "*kernel_trace*" -delete

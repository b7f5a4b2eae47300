#!/bin/bash
# Kernel trace of the default bench with host phase marks (no syncs), reduced on the box to the GPU idle
# time inside the timed window by host phase (tools/window_gaps.py).  Usage: tools/prof_window.sh <tag> [bench args]
set -e
TAG=${1:-run}; shift || true
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$R/gpurun_out/$TAG/marks.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pw_$TAG -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench.log 2>&1
python3 $R/tools/window_gaps.py $R/gpurun_out/pw_$TAG/run_kernel_trace.csv $TB_PHASE_MARKS > $R/gpurun_out/$TAG/window_gaps.txt
python3 $R/tools/kstats.py $R/gpurun_out/pw_$TAG/run_kernel_stats.csv > $R/gpurun_out/$TAG/kernel_stats.txt
rm -rf $R/gpurun_out/pw_$TAG
echo WINDOW_OK
tail -1 $R/gpurun_out/$TAG/bench.log | cut -c1-300
cat $R/gpurun_out/$TAG/window_gaps.txt

#!/bin/bash
# PyTorch-native / runtime kernel time inside the bench's timed window, attributed to the launching host phase
# (tools/window_native.py).  Usage: tools/prof_native.sh <tag> [bench args]
set -e
TAG=${1:-run}; shift || true
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$R/gpurun_out/$TAG/marks.json
timeout -k 10 700 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/pn_$TAG -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench.log 2>&1
python3 $R/tools/window_native.py /tmp/pn_$TAG/run_kernel_trace.csv $TB_PHASE_MARKS /tmp/pn_$TAG/run_hip_api_trace.csv > $R/gpurun_out/$TAG/window_native.txt
rm -rf /tmp/pn_$TAG
echo NATIVE_OK
cat $R/gpurun_out/$TAG/window_native.txt

#!/bin/bash
# Kernel time per sweep phase of the default bench (phases synchronised: TB_PHASE_TIMING=1), reduced on the box
# (tools/phase_kernels.py from the second timed step on).  Usage: tools/prof_phase_kernels.sh <tag> [bench args]
set -e
TAG=${1:-run}; shift || true
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_TIMING=1 TB_PHASE_MARKS=$R/gpurun_out/$TAG/phase_marks.json
timeout -k 10 700 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pk_$TAG -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench_phases.log 2>&1
FIRST=$(python3 -c "import json;m=json.load(open('$TB_PHASE_MARKS'));print([i for i,x in enumerate(m) if x[0].startswith('step')][1])")
python3 $R/tools/phase_kernels.py $R/gpurun_out/pk_$TAG/run_kernel_trace.csv $TB_PHASE_MARKS $FIRST > $R/gpurun_out/$TAG/phase_kernels.txt
rm -rf $R/gpurun_out/pk_$TAG
echo PHASE_KERNELS_OK
cat $R/gpurun_out/$TAG/phase_kernels.txt

#!/bin/bash
# Kernel trace of a short bench run, reduced on the box to the GEMM-role summary (tools/gemm_roles.py) and the
# kernel stats; the raw trace is deleted (hundreds of MB).   Usage: tools/prof_roles.sh <tag> [bench args...]
set -e
TAG=${1:-run}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/roles_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py "$@" > $O/bench.log 2>&1
T=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/gemm_roles.py $T > $O/roles.txt
find $O -name "*kernel_trace*" -delete
echo ROLES_OK
head -20 $O/roles.txt

#!/bin/bash
# A/B an environment toggle on the default bench: tools/gpu_ab.sh VAR val1 val2 [bench args]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; shift 3
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for V in $A $B; do
  env $VAR=$V timeout -k 10 500 python bench.py "$@" > gpurun_out/bench_ab_$V.log 2>&1
  tail -1 gpurun_out/bench_ab_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$V', d['value'], d['ms_per_step'])"
done

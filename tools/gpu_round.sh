#!/bin/bash
# One GPU pass on a fresh MI355X box: GPU test tier, smoke, default bench, then (optionally) a
# rocprofv3 kernel-stats profile of the bench.  Every GPU step has its own time limit; the first
# failing step ends the script (set -e).
# Usage: tools/gpu_round.sh <tag> [prof] [bench args...]
set -e
TAG=${1:-sanity}; shift || true
PROF=0
if [ "$1" = "prof" ]; then PROF=1; shift; fi
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 $OUT/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1
echo SMOKE_OK; tail -1 $OUT/smoke.log | cut -c1-300
timeout -k 10 600 python bench.py "$@" > $OUT/bench.log 2>&1
echo BENCH_OK; tail -1 $OUT/bench.log
if [ $PROF = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py "$@" --steps 4 --warmup 2 > $R/$OUT/prof_bench.log 2>&1
  echo PROF_OK
  find $R/$OUT/prof -name "*kernel_trace*" -delete
  python3 $R/tools/kstats.py $(find $R/$OUT/prof -name "*kernel_stats.csv" | head -1) 40 > $R/$OUT/kernel_stats.txt 2>&1 || true
  head -30 $R/$OUT/kernel_stats.txt
  python3 $R/tools/gemm_share.py $(find $R/$OUT/prof -name "*kernel_stats.csv" | head -1) > $R/$OUT/gemm_share.txt 2>&1 || true
  cat $R/$OUT/gemm_share.txt
fi

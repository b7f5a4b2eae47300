#!/bin/bash
# Bench A/B of the decode row-bucket granularity above 256 rows (TB_BUCKET_GRAN).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 256 128 64; do
  TB_BUCKET_GRAN=$g timeout -k 10 400 python bench.py > gpurun_out/bench_gran$g.log 2>&1
  echo "GRAN $g"; tail -1 gpurun_out/bench_gran$g.log | cut -c1-120
done

#!/bin/bash
# Fused vocab head vs hipBLASLt logits + decode_head on HEAD, alternated twice on one box (8 timed steps).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/head_ab
for i in 1 2; do
for o in "" "--no-fused-head"; do
  t=$(echo "x$o" | tr -d ' -')
  timeout -k 10 500 python bench.py --steps 8 --warmup 2 $o > gpurun_out/head_ab/bench_${t}_$i.log 2>&1
  echo "OPT [$o] $i"; tail -1 gpurun_out/head_ab/bench_${t}_$i.log | cut -c60-100
done
done

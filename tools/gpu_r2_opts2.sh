#!/bin/bash
# Option A/B on HEAD (one box, 8 timed steps): default, --no-fused-head, --fused-geglu.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/opts2
for o in "" "--no-fused-head" "--fused-geglu"; do
  t=$(echo "x$o" | tr -d ' -')
  timeout -k 10 500 python bench.py --steps 8 --warmup 2 $o > gpurun_out/opts2/bench_$t.log 2>&1
  echo "OPT [$o]"; tail -1 gpurun_out/opts2/bench_$t.log | cut -c1-130
done

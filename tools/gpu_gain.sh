#!/bin/bash
# Divergence / non-degeneracy of the random model vs the post-norm init gain.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gain
for g in ${GAINS:-1 2 4 8}; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --pairs-per-step 30 --init-gain $g > gpurun_out/gain/g$g.log 2>&1
  echo "gain $g: $(tail -1 gpurun_out/gain/g$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["work"])')"
done

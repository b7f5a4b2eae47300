#!/bin/bash
# Pairs per step 90 vs 100 (P100 seeded with the P90 TunableOp table), one box, 8 timed steps.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p100
for P in ${PLIST:-90 100 90 100}; do
  timeout -k 10 500 python bench.py --steps 8 --warmup 2 --pairs-per-step $P > gpurun_out/p100/bench_P${P}_$RANDOM.log 2>&1
  echo "P=$P"; tail -1 $(ls -t gpurun_out/p100/bench_P${P}_*.log | head -1) | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['work']['peak_mem_gb'])"
done

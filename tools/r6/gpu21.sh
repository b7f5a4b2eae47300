#!/bin/bash
# Session re-entry sanity on a fresh box: full GPU tier, then tb vs auto on one box (8 / 2 steps, no side sweeps)
set -o pipefail
O=gpurun_out/r6/s3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
S="--steps 8 --warmup 2 --no-lora-side --no-lowrank-side --no-post-forcing --no-config2"
timeout -k 10 400 python -u bench.py $S > $O/tb1.json 2> $O/tb1.err || exit 3
timeout -k 10 400 python -u bench.py $S --gemm auto > $O/auto1.json 2> $O/auto1.err || exit 4
timeout -k 10 400 python -u bench.py $S > $O/tb2.json 2> $O/tb2.err || exit 5
for f in tb1 auto1 tb2; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['work']['diverged_frac'])"; done

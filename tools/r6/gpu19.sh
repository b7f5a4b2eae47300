#!/bin/bash
# Round-end validation at HEAD: full GPU suite, smoke, default bench at the driver's shape (all side measurements)
set -o pipefail
O=gpurun_out/r6/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 3
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4

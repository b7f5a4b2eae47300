#!/bin/bash
set -o pipefail
O=gpurun_out/r6/full1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-post-forcing --no-config2 --no-lora-side --no-lowrank-side > $O/bench.json 2> $O/bench.err || exit 3

#!/bin/bash
set -o pipefail
O=gpurun_out/r6/lora2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --only-side lora --steps 4 --warmup 1 > $O/lora_split.json 2> $O/lora_split.err || exit 3

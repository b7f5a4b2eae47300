#!/bin/bash
# LoRA T with the K range split over a workgroup's waves: tests, then lora side split vs ring on one box
set -o pipefail
O=gpurun_out/r6/lorasplit; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --only-side lora --steps 6 --warmup 1 > $O/split1.json 2> $O/split1.err || exit 3
TB_LORA_T=ring timeout -k 10 400 python -u bench.py --only-side lora --steps 6 --warmup 1 > $O/ring1.json 2> $O/ring1.err || exit 4
timeout -k 10 400 python -u bench.py --only-side lora --steps 6 --warmup 1 > $O/split2.json 2> $O/split2.err || exit 5
TB_LORA_T=ring timeout -k 10 400 python -u bench.py --only-side lora --steps 6 --warmup 1 > $O/ring2.json 2> $O/ring2.err || exit 6

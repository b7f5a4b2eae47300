#!/bin/bash
set -o pipefail
O=gpurun_out/r6/lora; mkdir -p $O
timeout -k 10 600 python -u bench.py --only-side lora --steps 4 --warmup 1 > $O/lora_split.json 2> $O/lora_split.err || exit 2
TB_LORA_T_SPLIT=0 timeout -k 10 600 python -u bench.py --only-side lora --steps 4 --warmup 1 > $O/lora_ring.json 2> $O/lora_ring.err || exit 3

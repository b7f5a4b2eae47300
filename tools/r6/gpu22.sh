#!/bin/bash
# LoRA T in fixed K chunks (split / fold launch forms): tests, launch-form table, lora side with the B = 0 control
set -o pipefail
O=gpurun_out/r6/lorachunk; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || { tail -40 $O/pytest_lora.log; exit 2; }
tail -1 $O/pytest_lora.log
timeout -k 10 300 python -u tools/lora_t_bench.py > $O/lora_t.jsonl 2> $O/lora_t.err || { tail -20 $O/lora_t.err; exit 3; }
timeout -k 10 600 python -u bench.py --only-side lora --steps 6 --warmup 1 > $O/lora1.json 2> $O/lora1.err || { tail -20 $O/lora1.err; exit 4; }
cat $O/lora1.json

#!/bin/bash
# LoRA T tiles over all used columns + split policy: tests, launch-form table, lora side (+ B = 0 control) and headline
set -o pipefail
O=gpurun_out/r6/lorachunk2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || { tail -40 $O/pytest_lora.log; exit 2; }
tail -1 $O/pytest_lora.log
timeout -k 10 400 python -u tools/lora_t_bench.py > $O/lora_t.jsonl 2> $O/lora_t.err || { tail -20 $O/lora_t.err; exit 3; }
timeout -k 10 900 python -u bench.py --steps 8 --warmup 2 --no-lowrank-side --no-post-forcing --no-config2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['work']['diverged_frac'], json.dumps(d['lora']))"

#!/bin/bash
# ring two-source staging by a masked byte offset: LoRA tests (bit-exactness), two-source vs single-source timing
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s35; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || { tail -40 $O/pytest_lora.log; exit 2; }
tail -1 $O/pytest_lora.log
timeout -k 10 300 python -u tools/l2a_bench.py > $O/l2a.jsonl 2> $O/l2a.err || { tail -20 $O/l2a.err; exit 3; }
timeout -k 10 300 python -u tools/l2a_bench.py > $O/l2a_2.jsonl 2> $O/l2a_2.err || { tail -20 $O/l2a_2.err; exit 4; }
paste -d' ' <(cut -c1-120 $O/l2a.jsonl) <(python3 -c "import json; [print(json.loads(l)['ratio']) for l in open('$O/l2a_2.jsonl')]")

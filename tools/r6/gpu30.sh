#!/bin/bash
# ring two-source staging with a stage-level branch: bit-exactness tests, two-source vs single-source timing, lora
# side + equal-work control with the headline on one box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s30; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || { tail -40 $O/pytest_lora.log; exit 2; }
tail -1 $O/pytest_lora.log
timeout -k 10 300 python -u tools/l2a_bench.py > $O/l2a.jsonl 2> $O/l2a.err || { tail -20 $O/l2a.err; exit 3; }
cat $O/l2a.jsonl
timeout -k 10 900 python -u bench.py --steps 8 --warmup 2 --no-lowrank-side --no-post-forcing --no-config2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['lora']['forward_ms']), d['lora']['value'], d['lora']['control_b0'])"

#!/bin/bash
# one-wave decode attention register-budget variants: attention GPU tests, then per-variant timing + bit equality
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s32; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 2; }
tail -1 $O/pytest_attn.log
timeout -k 10 300 python -u tools/attn_bench.py --wave-variants --rows 256,1024,2048,4096,7260 > $O/attn_var.jsonl 2> $O/attn_var.err || { tail -20 $O/attn_var.err; exit 3; }
cat $O/attn_var.jsonl

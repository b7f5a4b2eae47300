#!/bin/bash
set -o pipefail
O=gpurun_out/r6/ab1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py tests/test_engine_gpu.py \
  > $O/pytest.log 2>&1 || exit 2
TB_EXACT_OUT=$O timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_exact_9b_gpu.py -k reuse \
  > $O/pytest_exact.log 2>&1 || exit 3
B="--steps 8 --warmup 2 --no-post-forcing --no-config2 --no-lora-side --no-lowrank-side"
timeout -k 10 400 python -u bench.py $B > $O/new1.json 2> $O/new1.err || exit 4
TB_GEMM_TABLE=configs/gemm_dispatch/gemma2-9b_r5.json timeout -k 10 400 python -u bench.py $B > $O/old1.json 2> $O/old1.err || exit 5
timeout -k 10 400 python -u bench.py $B > $O/new2.json 2> $O/new2.err || exit 6
TB_GEMM_TABLE=configs/gemm_dispatch/gemma2-9b_r5.json timeout -k 10 400 python -u bench.py $B > $O/old2.json 2> $O/old2.err || exit 7
timeout -k 10 600 python -u bench.py --only-side lora --steps 8 --warmup 2 > $O/lora.json 2> $O/lora.err || exit 8

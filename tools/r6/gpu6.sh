#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/bench gpurun_out/r6/exact
TB_EXACT_OUT=gpurun_out/r6/exact timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_exact_9b_gpu.py -k reuse > gpurun_out/r6/exact/pytest_exact_reuse.log 2>&1; r1=$?
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench/bench_20_5.json 2> gpurun_out/r6/bench/bench_20_5.err || exit 3
exit $r1

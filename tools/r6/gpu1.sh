#!/bin/bash
# round 6, first GPU call: memory size, full GPU suite, the 9B exactness and 2-rank bench tests
set -o pipefail
mkdir -p gpurun_out/r6
python -c "import torch; f,t=torch.cuda.mem_get_info(); print('free', f, 'total', t, 'props', torch.cuda.get_device_properties(0).total_memory)" > gpurun_out/r6/mem.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu \
  --ignore=tests/test_exact_9b_gpu.py --ignore=tests/test_bench_gpu.py > gpurun_out/r6/pytest_gpu.log 2>&1 || exit 2
TB_EXACT_OUT=gpurun_out/r6 timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_exact_9b_gpu.py tests/test_bench_gpu.py > gpurun_out/r6/pytest_9b.log 2>&1 || exit 3

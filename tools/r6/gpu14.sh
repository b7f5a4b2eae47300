#!/bin/bash
# random-basis kernel: kernel tests, projection-cell GPU tests, lowrank side measurement, its kernel profile
set -o pipefail
O=gpurun_out/r6/basis; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "random_basis or row_combine" > $O/pytest_k.log 2>&1 || exit 2
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_engine_gpu.py tests/test_exact_9b_gpu.py > $O/pytest.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --only-side lowrank --lowrank-steps 6 > $O/lowrank.json 2> $O/lowrank.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o lr -- python3 -u bench.py --only-side lowrank --lowrank-steps 2 > $O/lowrank_prof.json 2> $O/lowrank_prof.err || exit 4

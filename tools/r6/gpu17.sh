#!/bin/bash
# CGS2 random-basis kernel + vectorised lens-base terms: kernel tests, 9B exactness, lowrank side, headline profile
set -o pipefail
O=gpurun_out/r6/cgs2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "random_basis or row_combine" > $O/pytest_k.log 2>&1 || exit 2
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_exact_9b_gpu.py > $O/pytest_exact.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --only-side lowrank --lowrank-steps 6 > $O/lowrank.json 2> $O/lowrank.err || exit 4
bash tools/r6/prof_headline.sh head3 || exit 5

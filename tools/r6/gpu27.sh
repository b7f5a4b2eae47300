#!/bin/bash
# basis kernel load batching: bit-equality test, per-step workload timing per qu; lowrank side at the cell cap, twice
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s27; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k random_basis > $O/pytest_basis.log 2>&1 || { tail -30 $O/pytest_basis.log; exit 2; }
tail -1 $O/pytest_basis.log
timeout -k 10 300 python -u tools/basis_bench.py > $O/basis_bench.jsonl 2> $O/basis_bench.err || { tail -20 $O/basis_bench.err; exit 3; }
cat $O/basis_bench.jsonl

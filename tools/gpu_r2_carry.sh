#!/bin/bash
# Decode-tail carry-over with the cross-step pipeline: engine GPU tests, then bench A/B (carry 0 / 768 / 1536).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -1 gpurun_out/pytest_gpu.log
for C in 0 768 1536; do
  timeout -k 10 600 python bench.py --steps 8 --warmup 1 --carry-rows $C > gpurun_out/bench_carry$C.log 2>&1
  echo "carry=$C"; tail -1 gpurun_out/bench_carry$C.log | cut -c1-120; grep -o '"carried_cells_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*\|"pipelined_steps": [0-9]*' gpurun_out/bench_carry$C.log | tr '\n' ' '; echo
done

#!/bin/bash
# Refactored GEMM epilogue + fused head: full GPU tier, smoke, bench, and kernel stats of a short bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/head3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/head3/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/head3/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/head3/smoke.log 2>&1
echo SMOKE_OK; tail -1 gpurun_out/head3/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/head3/bench.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/head3/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/head3/pds -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/head3/bench_traced.log 2>&1
python3 $R/tools/decode_steps.py $R/gpurun_out/head3/pds/run_kernel_trace.csv > $R/gpurun_out/head3/decode_steps.txt
python3 $R/tools/kstats.py $R/gpurun_out/head3/pds/run_kernel_stats.csv 40 > $R/gpurun_out/head3/kernel_stats.txt
rm -f $R/gpurun_out/head3/pds/run_kernel_trace.csv
head -25 $R/gpurun_out/head3/kernel_stats.txt

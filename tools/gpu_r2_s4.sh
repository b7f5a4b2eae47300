#!/bin/bash
# Session-4 check on one MI355X: GPU test tier, smoke, default bench, then a kernel trace of a short bench
# with the per-decode-step / per-kernel-family breakdown (tools/decode_steps.py) and kernel stats.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/s4/pytest_gpu.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/s4/smoke.log 2>&1
echo SMOKE_OK; tail -1 gpurun_out/s4/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/s4/bench_default.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/s4/bench_default.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s4/pds -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/s4/bench_traced.log 2>&1
python3 $R/tools/decode_steps.py $R/gpurun_out/s4/pds/run_kernel_trace.csv > $R/gpurun_out/s4/decode_steps.txt
python3 $R/tools/kstats.py $R/gpurun_out/s4/pds/run_kernel_stats.csv 40 > $R/gpurun_out/s4/kernel_stats.txt
rm -f $R/gpurun_out/s4/pds/run_kernel_trace.csv
cat $R/gpurun_out/s4/decode_steps.txt
cd $R
timeout -k 10 400 python3 tools/hf_batched_baseline.py > gpurun_out/s4/hf_batched.log 2>&1
echo HFB_OK; tail -1 gpurun_out/s4/hf_batched.log

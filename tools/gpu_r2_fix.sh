#!/bin/bash
# Bench after the warmup/timed boundary fix: default (4 steps) and driver-shaped (20 steps, 5 warmup).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/fix
timeout -k 10 400 python bench.py > gpurun_out/fix/bench_default.log 2>&1
echo DEFAULT; tail -1 gpurun_out/fix/bench_default.log | cut -c1-140
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fix/bench_20_5.log 2>&1
echo LONG; tail -1 gpurun_out/fix/bench_20_5.log | cut -c1-140

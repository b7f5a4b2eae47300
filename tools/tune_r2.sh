#!/bin/bash
# Extend the TunableOp tables with the GEMM shapes of the current bench (P = 90, seeded with its table) and of a
# 120-pairs-per-step bench (seeded with the P90 table), then bench both with their tables.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop
cp configs/tunableop/gemma2-9b_P90_E4_new50.csv gpurun_out/tunableop/gemma2-9b_P90_E4_new50.csv
export TB_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tunableop
timeout -k 10 900 python bench.py --steps 4 --warmup 1 --tune-gemms > gpurun_out/tune_p90.log 2>&1 || echo "p90 tuning rc=$?"
cp gpurun_out/tunableop/gemma2-9b_P90_E4_new50.csv gpurun_out/tunableop/gemma2-9b_P120_E4_new50.csv
timeout -k 10 1000 python bench.py --steps 4 --warmup 1 --pairs-per-step 120 --tune-gemms > gpurun_out/tune_p120.log 2>&1 || echo "p120 tuning rc=$?"
wc -l gpurun_out/tunableop/*.csv
for P in 90 120; do
  timeout -k 10 600 python bench.py --steps 8 --warmup 1 --pairs-per-step $P > gpurun_out/bench_tuned_P$P.log 2>&1 || true
  echo "P=$P"; tail -1 gpurun_out/bench_tuned_P$P.log | cut -c1-160
done

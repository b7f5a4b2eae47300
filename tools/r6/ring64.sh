#!/bin/bash
# tb_shapes at the 64-row decode buckets: the batch-invariant variants at the row counts between the measured ones
set -o pipefail
mkdir -p gpurun_out/r6/gemm
MS=192,320,448,576,704,832,960,1088,1216,1344,1408,1472,1600,1664,1728,1856,1920,1984,2112,2240,2368,2496,2624,2752,2880,3008
timeout -k 10 1500 python -u tools/ring_bench.py --shapes o,down,qkv,gu --ms $MS --others g256,g128,gs --no-check --rounds 4 \
  --tiles 128x112,128x128,128x64,16x16,16x32,32x32,32x64,48x112,64x112,64x32,64x64,96x112,144x112,192x112,256x112 \
  --out gpurun_out/r6/gemm/ring64.jsonl > gpurun_out/r6/gemm/ring64.log 2>&1

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/bench
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench/bench_20_5_b.json 2> gpurun_out/r6/bench/bench_20_5_b.err || exit 3

#!/bin/bash
# add_rmsnorm2: one-wave-per-row kernel -- numerics test, microbenchmark, same-box bench A/B (TB_NORM_WAVE)
set -o pipefail
O=gpurun_out/r6/normwave; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm_family" > $O/pytest_k.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/norm_bench.py --rows 64,256,1024,4096,16384,32768 > $O/norm_bench.log 2>&1 || exit 3
B="python -u bench.py --steps 8 --warmup 2 --no-post-forcing --no-config2 --no-lora-side --no-lowrank-side"
TB_NORM_WAVE=1 timeout -k 10 300 $B > $O/wave1.json 2> $O/wave1.err || exit 4
timeout -k 10 300 $B > $O/block1.json 2> $O/block1.err || exit 5
TB_NORM_WAVE=1 timeout -k 10 300 $B > $O/wave2.json 2> $O/wave2.err || exit 6
timeout -k 10 300 $B > $O/block2.json 2> $O/block2.err || exit 7

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6/side
TB_PHASE_TIMING=1 timeout -k 10 600 python -u bench.py --only-side lowrank --lowrank-steps 3 --profile-steps > gpurun_out/r6/side/lowrank_prof.json 2> gpurun_out/r6/side/lowrank_prof.err || exit 2
timeout -k 10 600 python -u bench.py --only-side lora --steps 8 --warmup 2 > gpurun_out/r6/side/lora.json 2> gpurun_out/r6/side/lora.err || exit 3

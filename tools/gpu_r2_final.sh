#!/bin/bash
# Round-2 HEAD evidence: driver-shaped bench (20 timed / 5 warmup) and its --no-trie-decode / --no-skip-noop A/B
# on the same box, the 9B reference pipelines end to end, then a kernel-stats profile of the default bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/final
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_20_5.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/final/bench_20_5.log | cut -c1-200
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --no-trie-decode --no-skip-noop > gpurun_out/final/bench_20_5_plain.log 2>&1
echo BENCH_PLAIN_OK; tail -1 gpurun_out/final/bench_20_5_plain.log | cut -c1-200
bash tools/gpu_pipelines.sh > gpurun_out/final/pipelines.txt 2>&1
echo PIPES_OK; cat gpurun_out/final/pipelines.txt | grep -E "^run_|cells on"
bash tools/prof_stats.sh final_r2 > /dev/null
python3 tools/kstats.py gpurun_out/prof_final_r2/run_kernel_stats.csv > gpurun_out/final/kernel_stats.txt
head -25 gpurun_out/final/kernel_stats.txt

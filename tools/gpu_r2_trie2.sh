#!/bin/bash
# Prefix-trie decode: driver-shaped A/B (20 timed steps, 5 warmup; trie on / off), then a kernel-stats profile.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/trie
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/trie/bench_20_5_trie.log 2>&1
echo BENCH_TRIE; tail -1 gpurun_out/trie/bench_20_5_trie.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 --no-trie-decode > gpurun_out/trie/bench_20_5_notrie.log 2>&1
echo BENCH_NOTRIE; tail -1 gpurun_out/trie/bench_20_5_notrie.log
bash tools/prof_stats.sh trie

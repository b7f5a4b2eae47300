#!/bin/bash
# HEAD sanity after the prefix-trie decode + lens dedup: full GPU tier, smoke, driver-shaped bench, kernel stats.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trie
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/trie/pytest_all.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/trie/pytest_all.log
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/trie/smoke.log 2>&1
echo SMOKE_OK; tail -1 gpurun_out/trie/smoke.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/trie/bench_20_5.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/trie/bench_20_5.log
bash tools/prof_stats.sh trie

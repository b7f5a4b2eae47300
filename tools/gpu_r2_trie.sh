#!/bin/bash
# Prefix-trie decode: new GPU tests, then bench A/B (trie on / off) on one box.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trie
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fanout or trie or layer_resume or carry" > gpurun_out/trie/pytest.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/trie/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/trie/bench_trie.log 2>&1
echo BENCH_TRIE; tail -1 gpurun_out/trie/bench_trie.log
timeout -k 10 400 python bench.py --no-trie-decode > gpurun_out/trie/bench_notrie.log 2>&1
echo BENCH_NOTRIE; tail -1 gpurun_out/trie/bench_notrie.log

#!/bin/bash
# No-op spike skip (tails start at each cell's first effective spike): GPU tests, bench A/B on one box.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/noop
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/noop/pytest.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/noop/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/noop/bench_skip.log 2>&1
echo BENCH_SKIP; tail -1 gpurun_out/noop/bench_skip.log
timeout -k 10 400 python bench.py --no-skip-noop > gpurun_out/noop/bench_noskip.log 2>&1
echo BENCH_NOSKIP; tail -1 gpurun_out/noop/bench_noskip.log

set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 8 --warmup 1 > gpurun_out/bench_pipe.log 2>&1
echo BENCH_OK; tail -1 gpurun_out/bench_pipe.log | cut -c1-330
bash tools/prof_window.sh win2 --steps 4 --warmup 1

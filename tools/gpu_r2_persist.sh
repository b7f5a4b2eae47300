#!/bin/bash
# Persistent ping-pong GEMM: GPU numerics (incl. the persistent-vs-per-tile bit identity test), then the
# lab A/B (committed kernel vs tile-loop kernel with one workgroup per tile vs persistent grid).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/persist
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm_pp or vocab_head or lens_unembed" > gpurun_out/persist/pytest.log 2>&1
echo PYTEST_OK; tail -2 gpurun_out/persist/pytest.log
cd tools/lab && bash gemm_lab.sh run > ../../gpurun_out/persist/lab.log 2>&1
echo LAB_OK

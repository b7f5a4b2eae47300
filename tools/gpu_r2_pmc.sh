#!/bin/bash
# Round-2 PMC refresh of the hot kernels (incl. K/V fan-out, decode_head, the ping-pong SAE-encode GEMM).
set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc_kernels.sh
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc > $R/gpurun_out/pmc/pmc_hot_kernels.txt
# keep the summaries, drop bulky per-dispatch traces
find $R/gpurun_out/pmc -name "*kernel_trace*" -delete
cat $R/gpurun_out/pmc/pmc_hot_kernels.txt

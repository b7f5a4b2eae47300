#!/bin/bash
# PMC pass (SQ + GRBM counters, with kernel trace) over the lab GEMM variants and hipBLASLt at one shape.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_lab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SHAPE="4096 28672 3584"
CTR="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $O/$v -o run -- $R/tools/lab/gemm_lab_$v $SHAPE 0 5 > $O/$v.log 2>&1
  echo "$v OK"
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $O/hipblaslt -o run -- python3 $R/tools/lab/hipblaslt_gemm.py $SHAPE 8 > $O/hipblaslt.log 2>&1
echo "hipblaslt OK"

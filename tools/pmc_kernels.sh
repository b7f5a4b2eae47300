#!/bin/bash
# PMC counter passes over tools/pmc_kernels.py (hot kernels at the sweep's decode shapes).
# One block-limited counter set per pass (gfx950: <=8 SQ, <=4 TCC, <=2 GRBM), each pass its own
# time-limited run; kernel-trace stats in a separate run.  Writes gpurun_out/pmc/*.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/pmc_kernels.py > $O/plain.log 2>&1
echo PLAIN_OK; tail -1 $O/plain.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/pmc_kernels.py > $O/trace.log 2>&1
echo TRACE_OK
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/sq -o run -- python3 $R/tools/pmc_kernels.py > $O/sq.log 2>&1
echo SQ_OK
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/pmc_kernels.py > $O/fetch.log 2>&1
echo FETCH_OK
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/pmc_kernels.py > $O/write.log 2>&1
echo WRITE_OK

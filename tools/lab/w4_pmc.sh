#!/bin/bash
# PMC passes over the w4 lab binary (every kernel it times at one shape): tools/lab/w4_pmc.sh <build> [M N K]
set -e
R=$GRAFT_REPO_ROOT
B=$1; shift
SHAPE=${*:-4096 28672 3584}
O=$R/gpurun_out/w4_pmc_$B
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/p1 -o run -- $R/tools/lab/w4_lab_$B time $SHAPE 3 > $O/p1.log 2>&1
echo "p1 OK"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $O/p2 -o run -- $R/tools/lab/w4_lab_$B time $SHAPE 3 > $O/p2.log 2>&1
echo "p2 OK"

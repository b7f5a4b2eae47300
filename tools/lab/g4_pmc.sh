#!/bin/bash
# PMC passes (tools/lab/w4_pmc_parse.py) over g4_bench.py time at one shape: tools/lab/g4_pmc.sh <lib> <M,N,K>
set -e
R=$GRAFT_REPO_ROOT
LIB=$1; SHAPE=${2:-4096,28672,3584}
O=$R/gpurun_out/g4_pmc_${LIB%.so}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
export G4_LIB=$LIB G4_ROUNDS=2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/p1 -o run -- python3 $R/tools/lab/g4_bench.py time $SHAPE > $O/p1.log 2>&1
echo "p1 OK"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $O/p2 -o run -- python3 $R/tools/lab/g4_bench.py time $SHAPE > $O/p2.log 2>&1
echo "p2 OK"
python3 $R/tools/lab/w4_pmc_parse.py $O > $O/summary.txt
cat $O/summary.txt

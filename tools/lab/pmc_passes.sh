#!/bin/bash
# Counter passes over tools/lab/g4_bench.py at one shape (each pass its own run, --kernel-trace only):
#   tools/lab/pmc_passes.sh <lib.so> <tag> [M,N,K]      -> gpurun_out/pmc_<tag>/pN/run_counter_collection.csv
# then  python tools/lab/pmc_table.py gpurun_out/pmc_<tag>
set -e
R=$GRAFT_REPO_ROOT
LIB=$1; TAG=$2; SHAPE=${3:-4096,28672,3584}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export G4_LIB=$LIB G4_ROUNDS=2
PASSES=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE GRBM_COUNT"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"
 "SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD TCP_TCP_TA_ADDR_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_UTCL1_STALL_INFLIGHT_MAX TCP_TCC_READ_REQ TA_BUFFER_COALESCED_READ_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"
 "SQ_WAVE_CYCLES TCP_UTCL1_REQUEST TCP_UTCL1_SERIALIZATION_STALL TCP_TCR_TCP_STALL_CYCLES TCP_TD_TCP_STALL_CYCLES TA_BUFFER_READ_LDS_WAVEFRONTS TA_BUFFER_TOTAL_CYCLES"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/p$i -o run -- python3 $R/tools/lab/g4_bench.py time $SHAPE > $O/p$i.log 2>&1
  echo "pass $i OK"
done

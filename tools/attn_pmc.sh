#!/bin/bash
# Counter passes over the decode attention at the bench's shapes (tools/attn_bench.py, 4096 rows, shared-prefix
# layout), each pass its own run (--kernel-trace only), then the per-kernel table:
#   tools/attn_pmc.sh [tag]   -> gpurun_out/pmc_attn_<tag>/table.txt
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r5}
O=$R/gpurun_out/pmc_attn_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=(
 "FETCH_SIZE TCC_HIT_sum"
 "TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD"
 "SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TA_TA_BUSY"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/p$i -o run -- python3 $R/tools/attn_bench.py --rows 4096 --reps 5 > $O/p$i.log 2>&1
  echo "pass $i OK"
done
python3 $R/tools/lab/pmc_table.py $O > $O/table.txt
grep -A40 "attn_decode_wave" $O/table.txt | head -40

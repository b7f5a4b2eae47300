#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6/lora_prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for M in 64 2048; do for mode in lora base; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw_${M}_$mode -o run -- python3 $GRAFT_REPO_ROOT/tools/r6/lora_prof.py $M $mode > $O/log_${M}_$mode.txt 2>&1 || exit 2
  python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/raw_${M}_$mode/run_kernel_stats.csv > $O/kstats_${M}_$mode.txt || exit 3
  rm -rf $O/raw_${M}_$mode
done; done

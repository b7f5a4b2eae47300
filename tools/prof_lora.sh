#!/bin/bash
# Kernel stats of the bench with and without the unmerged LoRA bank (summaries only).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/lora
cd /tmp && export TMPDIR=/tmp
for opt in "" "--lora-rank 8"; do
  tag=$([ -z "$opt" ] && echo base || echo lora)
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pl -o run -- python3 $R/bench.py --steps 2 --pairs-per-step 60 $opt > $R/gpurun_out/lora/bench_$tag.log 2>&1
  python3 $R/tools/kstats.py $R/gpurun_out/pl/run_kernel_stats.csv > $R/gpurun_out/lora/kstats_$tag.txt
  rm -rf $R/gpurun_out/pl
  echo "$tag: $(tail -1 $R/gpurun_out/lora/bench_$tag.log | cut -c1-110)"
  head -14 $R/gpurun_out/lora/kstats_$tag.txt
done

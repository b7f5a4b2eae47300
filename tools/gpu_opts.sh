#!/bin/bash
# Bench options on one MI355X: unmerged LoRA bank, plain prefix-shared decode, decode-tail carry-over.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for opt in "--lora-rank 8" "--no-layer-resume" "--carry-rows 512"; do
  tag=$(echo $opt | tr -d ' -')
  timeout -k 10 400 python bench.py --steps 2 --pairs-per-step 60 $opt > gpurun_out/b_$tag.log 2>&1
  echo "$opt: $(tail -1 gpurun_out/b_$tag.log | cut -c1-130)"
done

#!/bin/bash
# The multi-adapter sweep through the CLI at 9B (configs/ablation_lora_bank.yaml: the 3 words' rank-8 adapters as one
# unmerged bank, fused into the in-tree GEMMs), SAE methods, DP = 1, with its wall time
set -o pipefail
R=gpurun_out/r6/pipelines_9b_lora
mkdir -p $R
t0=$(python3 -c "import time; print(time.time())")
timeout -k 10 900 python -m taboo_brittleness_amd run_sweep configs/ablation_lora_bank.yaml --methods sae \
  --set runtime.batch_size=8192 --out $R/results/sweeps/sae_lora_bank > $R/sweep_lora_bank.log 2>&1
rc=$?
t1=$(python3 -c "import time; print(time.time())")
echo "run_sweep_sae_lora_bank: rc=$rc $(python3 -c "print(round($t1 - $t0, 1))") s" | tee $R/summary.txt
tail -5 $R/sweep_lora_bank.log | tee -a $R/summary.txt
ls $R/results/sweeps/sae_lora_bank | tee -a $R/summary.txt
exit $rc

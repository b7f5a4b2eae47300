#!/bin/bash
# Reference entry points at full Gemma-2-9B size on one MI355X (BASELINE config 2 + SAE baseline +
# token forcing + a small sweep), with wall times.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pipes
R=gpurun_out/pipes
S() { python3 -c "import time; print(time.time())"; }
t0=$(S); timeout -k 10 600 python -m taboo_brittleness_amd run_generation configs/ll_baseline_9b.yaml --set data.processed_dir=$R/processed > $R/gen.log 2>&1; t1=$(S)
echo "run_generation: $(python3 -c "print(round($t1 - $t0, 1))") s"; tail -2 $R/gen.log
t0=$(S); timeout -k 10 600 python -m taboo_brittleness_amd reproduce_logit_lens configs/ll_baseline_9b.yaml --set data.processed_dir=$R/processed --set output.base_dir=$R/results/logit_lens > $R/ll.log 2>&1; t1=$(S)
echo "reproduce_logit_lens: $(python3 -c "print(round($t1 - $t0, 1))") s"; tail -3 $R/ll.log
t0=$(S); timeout -k 10 600 python -m taboo_brittleness_amd run_sae_baseline configs/ll_baseline_9b.yaml --set data.processed_dir=$R/processed --set data.results_dir=$R/results > $R/sae.log 2>&1; t1=$(S)
echo "run_sae_baseline: $(python3 -c "print(round($t1 - $t0, 1))") s"; tail -3 $R/sae.log
t0=$(S); timeout -k 10 600 python -m taboo_brittleness_amd run_token_forcing configs/ll_baseline_9b.yaml --mode postgame --set data.results_dir=$R/results > $R/tf.log 2>&1; t1=$(S)
echo "run_token_forcing postgame: $(python3 -c "print(round($t1 - $t0, 1))") s"; tail -3 $R/tf.log
t0=$(S); timeout -k 10 900 python -m taboo_brittleness_amd run_sweep configs/ll_baseline_9b.yaml --methods all --set runtime.batch_size=4096 --out $R/results/sweeps/all > $R/sweep.log 2>&1; t1=$(S)
echo "run_sweep (all methods): $(python3 -c "print(round($t1 - $t0, 1))") s"; tail -3 $R/sweep.log
# the npz caches / sweep shards are large: keep the logs and summaries only (gpurun copies back <= 64 MiB)
rm -rf $R/processed
find $R/results -name "*.npz" -delete

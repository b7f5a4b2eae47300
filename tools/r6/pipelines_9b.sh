#!/bin/bash
# Every reference entry point at full Gemma-2-9B size on one MI355X at HEAD, with wall times:
# run_generation, reproduce_logit_lens, run_sae_baseline (BASELINE config 2 + the SAE baseline), run_sweep with the
# SAE methods (config 3 at DP = 1) and the projection methods (config 4, ranks 1..64, at DP = 1), token forcing
# pregame / postgame (+ the config-5 shape TP = 2 as two processes sharing the GPU, one-shot P2P all-reduce),
# make_report.  Each step has its own time limit; the first failure ends the script.
set -o pipefail
R=gpurun_out/r6/pipelines_9b
mkdir -p $R
S() { python3 -c "import time; print(time.time())"; }
step() {   # name, limit, log, command...
  local name=$1 lim=$2 log=$3; shift 3
  local t0=$(S)
  timeout -k 10 $lim "$@" > $R/$log 2>&1
  local rc=$?
  local t1=$(S)
  echo "$name: rc=$rc $(python3 -c "print(round($t1 - $t0, 1))") s" | tee -a $R/summary.txt
  tail -3 $R/$log >> $R/summary.txt
  return $rc
}
: > $R/summary.txt
step run_generation 600 gen.log python -m taboo_brittleness_amd run_generation configs/ll_baseline_9b.yaml \
  --set data.processed_dir=$R/processed || exit 1
step reproduce_logit_lens 600 ll.log python -m taboo_brittleness_amd reproduce_logit_lens configs/ll_baseline_9b.yaml \
  --set data.processed_dir=$R/processed --set output.base_dir=$R/results/logit_lens || exit 2
step run_sae_baseline 600 sae.log python -m taboo_brittleness_amd run_sae_baseline configs/ll_baseline_9b.yaml \
  --set data.processed_dir=$R/processed --set data.results_dir=$R/results || exit 3
step run_sweep_sae_config3 900 sweep_sae.log python -m taboo_brittleness_amd run_sweep configs/ablation_dp4.yaml \
  --methods sae --set parallel.dp=1 --set runtime.batch_size=8192 --out $R/results/sweeps/sae || exit 4
step run_sweep_proj_config4 900 sweep_proj.log python -m taboo_brittleness_amd run_sweep configs/lowrank_dp8.yaml \
  --methods proj --set parallel.dp=1 --set runtime.batch_size=8192 --out $R/results/sweeps/proj || exit 5
step run_token_forcing_pregame 600 tf_pre.log python -m taboo_brittleness_amd run_token_forcing \
  configs/ll_baseline_9b.yaml --mode pregame --set data.results_dir=$R/results || exit 6
step run_token_forcing_postgame 600 tf_post.log python -m taboo_brittleness_amd run_token_forcing \
  configs/ll_baseline_9b.yaml --mode postgame --set data.results_dir=$R/results || exit 7
step run_token_forcing_tp2_p2p 600 tf_tp2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29811 -m taboo_brittleness_amd.cli.run_token_forcing configs/forcing_tp2dp4.yaml \
  --mode postgame --set parallel.dp=1 --set parallel.backend=gloo --set data.results_dir=$R/results_tp2 || exit 8
step make_report 300 report.log python -m taboo_brittleness_amd make_report --results $R/results --out $R/results/figures \
  || exit 9
# the npz caches / sweep shards are large: keep logs, summaries and result JSON / CSV only
rm -rf $R/processed
find $R -name "*.npz" -delete
find $R -path "*parts_*" -delete 2>/dev/null
find $R -name "shard_*.json" -delete
find $R -name "sweep_cells.jsonl" -size +20M -delete
exit 0

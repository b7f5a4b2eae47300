#!/bin/bash
# Round-6 final validation at HEAD: GPU test tier, smoke, driver-shape bench (20 / 5, every side measurement incl.
# the lora B = 0 control), then a kernel census of the lora side (4 / 1 steps, control off).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/${FINAL_TAG:-final2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log | cut -c1-300
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['work']['diverged_frac'], d['mem']['peak_hbm_frac'], d['lora']['value'], d['lora'].get('control_b0'), d['lowrank']['value'], d['post_forcing']['settings_per_s'], d['config2']['pairs_per_s'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_lora -o run -- python3 $R/bench.py --only-side lora --steps 4 --warmup 1 --no-lora-control > $R/$O/prof_lora_bench.json 2> $R/$O/prof_lora_bench.err || exit 5
find $R/$O/prof_lora -name "*kernel_trace*" -delete
python3 $R/tools/kstats.py $(find $R/$O/prof_lora -name "*kernel_stats.csv" | head -1) 40 > $R/$O/kernel_stats_lora.txt 2>&1 || true
head -25 $R/$O/kernel_stats_lora.txt

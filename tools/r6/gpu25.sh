#!/bin/bash
# LoRA tests + T launch table after the fold-kernel change; lowrank side (BASELINE config 4): timed-window kernel
# census and GPU idle by host phase
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s25; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lora_gpu.py > $O/pytest_lora.log 2>&1 || { tail -40 $O/pytest_lora.log; exit 2; }
tail -1 $O/pytest_lora.log
timeout -k 10 400 python -u tools/lora_t_bench.py > $O/lora_t.jsonl 2> $O/lora_t.err || { tail -20 $O/lora_t.err; exit 3; }
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$R/$O/marks_lowrank.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/raw -o run -- python3 $R/bench.py --only-side lowrank --lowrank-steps 4 > $R/$O/lowrank.json 2> $R/$O/lowrank.err || exit 4
W=$(python3 -c "import json; d=json.load(open('$R/$O/lowrank.json')); print(round(d['ms_per_step']*4/1000, 2))")
python3 $R/tools/window_kstats.py $R/$O/raw/run_kernel_trace.csv $W > $R/$O/kernel_stats_lowrank_timed.txt || exit 5
python3 $R/tools/window_gaps.py $R/$O/raw/run_kernel_trace.csv $TB_PHASE_MARKS > $R/$O/window_gaps_lowrank.txt || true
rm -rf $R/$O/raw
head -3 $R/$O/window_gaps_lowrank.txt; head -25 $R/$O/kernel_stats_lowrank_timed.txt

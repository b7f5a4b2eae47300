#!/bin/bash
# Timed-window kernel census of the headline bench (4 timed / 2 warmup steps, side measurements off).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/prof/${1:-head}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$O/marks.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $R/bench.py \
  --steps 4 --warmup 2 --no-post-forcing --no-config2 --no-lora-side --no-lowrank-side > $O/bench.json 2> $O/bench.err || exit 2
W=$(python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['ms_per_step']*4/1000, 2))")
python3 $R/tools/window_kstats.py $O/raw/run_kernel_trace.csv $W > $O/kernel_stats_timed.txt || exit 3
python3 $R/tools/window_gaps.py $O/raw/run_kernel_trace.csv $TB_PHASE_MARKS > $O/window_gaps.txt || true
rm -rf $O/raw

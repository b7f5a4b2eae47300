#!/bin/bash
# pooled PCA bases on the device + batched basis-kernel loads: full GPU tier, then the lowrank side's timed-window
# census and GPU idle (vs gpurun_out/r6/s25)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r6/s26; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
export TB_PHASE_MARKS=$R/$O/marks_lowrank.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/raw -o run -- python3 $R/bench.py --only-side lowrank --lowrank-steps 4 > $R/$O/lowrank.json 2> $R/$O/lowrank.err || exit 4
W=$(python3 -c "import json; d=json.load(open('$R/$O/lowrank.json')); print(round(d['ms_per_step']*4/1000, 2))")
python3 $R/tools/window_kstats.py $R/$O/raw/run_kernel_trace.csv $W > $R/$O/kernel_stats_lowrank_timed.txt || exit 5
python3 $R/tools/window_gaps.py $R/$O/raw/run_kernel_trace.csv $TB_PHASE_MARKS > $R/$O/window_gaps_lowrank.txt || true
rm -rf $R/$O/raw
cat $R/$O/lowrank.json; head -12 $R/$O/window_gaps_lowrank.txt; grep -E "random_basis|GEMMs|window" $R/$O/kernel_stats_lowrank_timed.txt
cd $R
timeout -k 10 400 python3 bench.py --only-side lowrank --lowrank-steps 4 --side-pairs 120 > $O/lowrank_p120.json 2> $O/lowrank_p120.err || exit 6
timeout -k 10 400 python3 bench.py --only-side lowrank --lowrank-steps 4 > $O/lowrank_auto.json 2> $O/lowrank_auto.err || exit 7
cat $O/lowrank_p120.json; echo; cat $O/lowrank_auto.json

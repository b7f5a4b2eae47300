#!/bin/bash
# Final profiles of the default bench, summarised on the box (kernel traces are too big to ship back):
# rocprofv3 kernel stats + GPU idle gaps, then per-phase kernel attribution (phases synchronised).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-post-forcing --no-config2 > $R/gpurun_out/final/bench_rocprof.log 2>&1
python3 $R/tools/kstats.py $R/gpurun_out/pf/run_kernel_stats.csv > $R/gpurun_out/final/kernel_stats.txt
python3 $R/tools/gaps.py $R/gpurun_out/pf/run_kernel_trace.csv 6.0 > $R/gpurun_out/final/gpu_gaps_timed.txt
T=$(python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(d['steps'] * d['ms_per_step'] / 1e3)" $R/gpurun_out/final/bench_rocprof.log)
python3 $R/tools/window_kstats.py $R/gpurun_out/pf/run_kernel_trace.csv $T > $R/gpurun_out/final/kernel_stats_timed.txt
cp $R/gpurun_out/pf/run_kernel_stats.csv $R/gpurun_out/final/kernel_stats.csv
rm -rf $R/gpurun_out/pf
export TB_PHASE_TIMING=1 TB_PHASE_MARKS=$R/gpurun_out/final/phase_marks.json
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pp -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-post-forcing --no-config2 > $R/gpurun_out/final/bench_phases.log 2>&1
python3 $R/tools/phase_kernels.py $R/gpurun_out/pp/run_kernel_trace.csv $R/gpurun_out/final/phase_marks.json 35 > $R/gpurun_out/final/phase_kernels_last_step.txt
rm -rf $R/gpurun_out/pp
echo FINAL_PROF_OK
head -12 $R/gpurun_out/final/kernel_stats.txt
cat $R/gpurun_out/final/phase_kernels_last_step.txt

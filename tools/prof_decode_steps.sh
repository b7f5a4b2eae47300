set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ds
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pds -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/ds/bench.log 2>&1
python3 $R/tools/decode_steps.py $R/gpurun_out/pds/run_kernel_trace.csv > $R/gpurun_out/ds/decode_steps.txt
rm -rf $R/gpurun_out/pds
cat $R/gpurun_out/ds/decode_steps.txt

set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof3.log 2>&1
echo PROF_OK
find $R/gpurun_out/prof3 -name "*stats*"

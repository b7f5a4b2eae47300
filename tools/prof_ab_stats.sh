#!/bin/bash
# Kernel stats of the bench under two env settings (A/B), summarised on the box.
# Usage: tools/prof_ab_stats.sh <tag> "<envA>" "<envB>" [bench args]
set -e
TAG=$1; EA=$2; EB=$3; shift 3
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for arm in A B; do
  if [ $arm = A ]; then E="$EA"; else E="$EB"; fi
  env $E true
  ( export $E; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$arm -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench_$arm.log 2>&1 )
  python3 $R/tools/kstats.py $R/gpurun_out/ab_$arm/run_kernel_stats.csv > $R/gpurun_out/$TAG/kstats_$arm.txt
  rm -rf $R/gpurun_out/ab_$arm
  echo "== $arm ($E)"; head -14 $R/gpurun_out/$TAG/kstats_$arm.txt
done

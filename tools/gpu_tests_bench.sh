#!/bin/bash
# GPU test files given as $TESTS (default: the whole gpu tier), then optional benches given as
# "tag:args" pairs in $BENCHES (each its own time limit).  First failure ends the script.
set -e
R=$GRAFT_REPO_ROOT; cd $R
OUT=gpurun_out/${TAG:-tb}; mkdir -p $OUT
if [ -n "$TESTS" ] || [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 200 --timeout-method thread $PYTEST_ARGS > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASS|FAIL|ERROR" $OUT/pytest.log | tail -30; [ -n "$KEEP_GOING" ] || exit 1; }
  echo PYTEST_DONE; tail -2 $OUT/pytest.log
fi
for b in $BENCHES; do
  tag=${b%%:*}; args=${b#*:}; args=${args//,/ }
  timeout -k 10 600 python bench.py $args > $OUT/bench_$tag.log 2>&1
  echo "BENCH $tag"; tail -1 $OUT/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['work']['diverged_frac'], d['config'].get('gemm_dispatch'))"
done

#!/bin/bash
# One GPU session: the -m gpu parity suite, smoke(), then the default bench
# line; each step under its own limit, stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
nproc > $OUT/nproc.txt; lscpu > $OUT/lscpu.txt 2>&1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.json; [ $rc -ne 0 ] && exit $rc
fi
exit 0

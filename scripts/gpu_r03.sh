#!/bin/bash
# round 3 GPU session: parity suite, then the legs named in $LEGS
# (bench.py --only <leg>), each under its own time limit; stops at the first
# failure. Usage: gpurun -- bash scripts/gpu_r03.sh [leg ...]
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
nproc > $OUT/nproc.txt; lscpu > $OUT/lscpu.txt 2>&1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
fi
for leg in "$@"; do
  timeout -k 10 600 python -u bench.py --only $leg $BENCH_ARGS > $OUT/leg_$leg.json 2> $OUT/leg_$leg.err
  rc=$?; echo "leg $leg rc=$rc"; tail -c 1500 $OUT/leg_$leg.json; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0

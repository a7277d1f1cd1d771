#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that ends in anything but success / test failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step tests 900 python -m pytest tests/test_gpu_parity.py -q -rf --timeout 600
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 900 python bench.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step prof_em 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_em" -o em -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-extra --no-cpu --steps 20 --warmup 5
  step prof_ck 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ck" -o ck -- python3 "$GRAFT_REPO_ROOT/bench.py" --only cksum --steps 20 --warmup 3
fi
echo done >> "$OUT/steps.log"

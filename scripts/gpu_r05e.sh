#!/bin/bash
# Round 5: the ring sweep with native submitter threads (bg_ring_run_lanes),
# the pooled plugin legs again, the ring ticket stamps at 16 submitters.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05e"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ring.py
step sweep 600 python -u bench.py --only sweep --steps 5 --warmup 2
step trace 300 python -u scripts/ring_trace.py --batch=4096 4 16
step pool 600 python -u bench.py --only plugin_pool
echo done >> "$OUT/steps.log"

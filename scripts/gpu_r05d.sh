#!/bin/bash
# Round 5: zero-copy checksum pipes (host-registered packet pool) parity and
# the pooled plugin legs; where the 16-submitter ring sweep's time goes
# (per-ticket stamps, A/B build).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05d"
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
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pipe.py tests/test_bessd_wrappers.py \
  "tests/test_gpu_parity.py::test_wm_tags_fewer_direct_tuples"
step pool 600 python -u bench.py --only plugin_pool
step trace 300 python -u scripts/ring_trace.py --batch=4096 4 16
step trace512 300 python -u scripts/ring_trace.py --batch=512 4 16
echo done >> "$OUT/steps.log"

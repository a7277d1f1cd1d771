#!/bin/bash
# Round 5: WildcardMatch parity (unused direct slots; streamed and not),
# the tag-word kernel's phases streamed / not (A/B build), the ring sweep
# with sleeping waits.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05c"
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
step dbg 180 python -u scripts/dbg_wm_staged.py
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pipe.py tests/test_attr_fields.py
step phase 600 python -u scripts/variants.py wmphase
step sweep 600 python -u bench.py --only sweep --steps 5 --warmup 2
echo done >> "$OUT/steps.log"

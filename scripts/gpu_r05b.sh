#!/bin/bash
# Round 5: WildcardMatch staged-row diagnosis; the streamed tag-word kernel's
# parity (run-time compiled and ahead-of-time, streamed or not) and its
# C4 times; the pooled plugins with the pipe's per-call launch times.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05b"
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
  tests/test_wm_jit.py "tests/test_gpu_configs.py::test_c4_imix_2k_slots" \
  "tests/test_gpu_configs.py::test_c4_header_slab_full_size"
step wm 300 python -u bench.py --only wm --no-cpu --steps 20 --warmup 5
step pool 600 python -u bench.py --only plugin_pool
echo done >> "$OUT/steps.log"

#!/bin/bash
# Round 5: checksum words-only form as the default (parity + A/B), the
# streamed WildcardMatch form at producer depth 24 (64-entry consumer queues)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05j"
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
step tests 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_wm_jit.py tests/test_gpu_configs.py tests/test_gpu_pipe.py
step forms 300 python -u scripts/ck_forms_parity.py
step ck 600 python -u scripts/variants.py ck
step wmstream 600 python -u scripts/variants.py wmstream
step wm 600 python -u bench.py --only wm --no-cpu
step c3 300 python -u bench.py --only cksum --no-cpu
step probe 300 ./scripts/bin/hbm_probe 2 c
echo done >> "$OUT/steps.log"

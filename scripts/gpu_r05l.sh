#!/bin/bash
# Round 5: WildcardMatch slot records (key + value in one 32 B record) and
# the two-byte direct-tuple policy: parity, then C4's legs
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05l"
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
step tests 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_wm_jit.py tests/test_gpu_configs.py tests/test_gpu_pipe.py tests/test_gpu_ring.py
step wm 600 python -u bench.py --only wm --no-cpu
step wmdirect 600 python -u scripts/variants.py wmdirect
step wmstream 600 python -u scripts/variants.py wmstream
echo done >> "$OUT/steps.log"

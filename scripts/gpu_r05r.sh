#!/bin/bash
# Round 5: WildcardMatch line form (dense 64 B slots, whole-line tile loads)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05r"
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
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_wm_jit.py tests/test_gpu_configs.py tests/test_gpu_ring.py tests/test_gpu_pipe.py tests/test_bessd_wrappers.py
step wm 600 python -u bench.py --only wm --no-cpu
step wmstream 600 python -u scripts/variants.py wmstream
echo done >> "$OUT/steps.log"

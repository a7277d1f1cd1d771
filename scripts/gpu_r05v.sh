#!/bin/bash
# Round 5: workgroups per CU for the read-only line ops; the new NAT / line
# op grids re-measured
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05v"
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
step lineocc 300 python -u scripts/variants.py lineocc
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dnat.py tests/test_static_nat.py tests/test_update_ttl.py tests/test_gpu_hashlb.py
echo done >> "$OUT/steps.log"

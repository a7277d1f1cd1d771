#!/bin/bash
# Round 5: A/B of the EM kernels -- 1500 B pair loads vs lane kernel, C5's
# sequential second-bucket lookup, C2's nontemporal gate stores
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05m"
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
step em1500 300 python -u scripts/variants.py em1500
step c5 600 python -u scripts/variants.py c5
step em 600 python -u scripts/variants.py em
echo done >> "$OUT/steps.log"

#!/bin/bash
# Round 5: blocked second bucket (both tag words in one line): every GPU
# test, C5 / NAT variants, and the bench as the driver runs it
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05q"
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
step tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step c5 600 python -u scripts/variants.py c5
step nat 300 python -u scripts/variants.py natphase
step bench 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo done >> "$OUT/steps.log"

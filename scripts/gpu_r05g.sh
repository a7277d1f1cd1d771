#!/bin/bash
# Round 5 full session: every GPU test, smoke, the bench line, the bench's
# kernel trace (rocprofv3 --kernel-trace --stats).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05g"
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
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -rf
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python -u bench.py --steps 20 --warmup 5
step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-e2e --steps 20 --warmup 5
echo done >> "$OUT/steps.log"

#!/bin/bash
# Round 5 closing call: every GPU test, smoke, the bench as the driver runs
# it and with the defaults, the kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/${OUTDIR:-r05s}"
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
step bench 900 python3 bench.py
step prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-e2e
echo done >> "$OUT/steps.log"

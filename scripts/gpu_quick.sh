#!/bin/bash
# tests + variants + bench on one box
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc" >> "$OUT/steps.log"; if [ $rc -gt 1 ]; then exit $rc; fi; }
rocm-smi --showclocks > "$OUT/clocks.txt" 2>&1 || true
run tests 900 python -m pytest tests -m gpu -q -rf --timeout 600
run variants 900 python scripts/variants.py ${VARIANTS:-em,ck}
run bench 900 python bench.py ${BENCH_ARGS:-}

#!/bin/bash
# The headline (C2) at the driver's step count against a long run, and with
# a longer settle, interleaved in one call:
#   gpurun -- bash scripts/headline_steps.sh OUTDIR
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"
mkdir -p "$OUT"
for rep in 1 2; do
  for A in "--steps 20 --warmup 5" "--steps 200 --warmup 20" "--steps 20 --warmup 5 --settle-ms 500"; do
    tag=$(echo "$A" | tr -d ' -')
    timeout -k 10 300 python bench.py --no-extra --no-cpu $A > "$OUT/h_${tag}_$rep.out" 2> "$OUT/h_${tag}_$rep.err" || exit $?
  done
done

#!/bin/bash
# Same-box A/B of library builds: [AB_ARGS=...] scripts/ab_libs.sh SCRIPT LIB1 LIB2 ...
# runs `python SCRIPT LIB $AB_ARGS` for each library twice (interleaved),
# each under its own time limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
S=$1; shift
for rep in 1 2; do
  for L in "$@"; do
    timeout -k 10 180 python "$S" "$L" $AB_ARGS >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "fail $L rc=$?" >> "$OUT/ab.err"; exit 3; }
  done
done

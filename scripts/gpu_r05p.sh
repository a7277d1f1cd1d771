#!/bin/bash
# Round 5: the bench as the driver runs it (--steps 20 --warmup 5)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05p"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
echo "rc=$?" >> "$OUT/steps.log"

#!/bin/bash
# round 4: GPU tests, the pool-bounded plugin leg, WM quad-load A/B
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --only plugin_pool > $OUT/pp.json 2> $OUT/pp.err || exit $?
for q in 1 0 1 0; do
  BG_WM_QUAD=$q WM_AB_FLAGS=512 timeout -k 10 200 python scripts/wm_ab.py scripts/bin/libbessgpu_ab.so >> $OUT/wmq.jsonl 2>> $OUT/wmq.err || exit $?
done

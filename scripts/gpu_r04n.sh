#!/bin/bash
# round 4: C4 pair loads on the 2 KB slots (A/B build, BG_WM_PAIR_ANY), two reps
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for rep in 1 2; do
  for k in 0 1; do
    BG_WM_PAIR_ANY=$k timeout -k 10 300 python scripts/wm_ab.py scripts/bin/libbessgpu_ab.so | sed "s/^{/{\"pair_any\": $k, /" >> $OUT/wm_pair.jsonl 2>> $OUT/wm_pair.err || exit $?
  done
done

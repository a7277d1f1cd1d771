#!/bin/bash
# round 4: WildcardMatch plugin on the bounded pool -- steady state
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for nw in 16 1; do
  timeout -k 10 240 python scripts/plugin_wm_repro.py 100000 "pool 262144" "pipeline $nw 1 0 0 0" "sleep 3000" "pipeline $nw 40 0 0 0" > $OUT/wmpool_$nw.txt 2>&1 || exit $?
done

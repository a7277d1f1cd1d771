#!/bin/bash
# round 4: WildcardMatch plugin slot sizes on the bounded pool (A/B drives)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for d in tests/bessd_shell/build/drive scripts/bin/drive_wm_512x8 scripts/bin/drive_wm_256x8 scripts/bin/drive_wm_256x16; do
  DRIVE=$d timeout -k 10 400 python scripts/pool_scaling.py 8 16 >> $OUT/pool_sizes.jsonl 2>> $OUT/pool_sizes.err || exit $?
done

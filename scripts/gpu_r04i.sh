#!/bin/bash
# round 4: bounded-pool plugin leg (Sources copy frame lengths, magazine pool)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bessd_wrappers.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t8.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --only plugin_pool > $OUT/pp8.json 2> $OUT/pp8.err || exit $?
timeout -k 10 240 python scripts/plugin_wm_repro.py 100000 "pool 262144" "pipeline 16 1 0 0 0" "pipeline 16 40 0 0 0" > $OUT/wmpool_16.txt 2>&1 || exit $?

#!/bin/bash
# round 4: run-time compiles in the bg_rtc helper process -- the GPU suite,
# then the bounded-pool plugin leg
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t10.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --only plugin_pool > $OUT/pp10.json 2> $OUT/pp10.err || exit $?

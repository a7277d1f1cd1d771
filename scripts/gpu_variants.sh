#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -rf --timeout 500 > "$OUT/tests.out" 2>&1
rc=$?; echo "tests rc=$rc" > "$OUT/steps.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/variants.py em,ck,wm > "$OUT/variants.json" 2> "$OUT/variants.err"
rc=$?; echo "variants rc=$rc" >> "$OUT/steps.log"; exit $rc

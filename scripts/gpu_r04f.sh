#!/bin/bash
# round 4: ring ticket runs -- mixed-run parity, e2e pipe / plugin legs
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t7.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --only pipe > $OUT/pipe7.json 2> $OUT/pipe7.err || exit $?
timeout -k 10 600 python bench.py --only plugin > $OUT/plugin7.json 2> $OUT/plugin7.err || exit $?

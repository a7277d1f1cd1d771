#!/bin/bash
# round 4: WildcardMatch ring -- pipe / plugin / module tests, pool leg
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_bessd_wrappers.py tests/test_gpu_ring.py tests/test_wm_jit.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t12.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --only plugin_pool > $OUT/pp14.json 2> $OUT/pp14.err || exit $?
timeout -k 10 900 python bench.py --only pipe > $OUT/pipe14.json 2> $OUT/pipe14.err || exit $?

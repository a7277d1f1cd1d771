#!/bin/bash
# round 4: WildcardMatch header prefetch issued after the tile's key loads --
# WM parity tests, then an A/B of bench.py --only wm (both layouts) against
# the previous tree's library (scripts/bin/prev), alternating, two reps
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_wm_jit.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ring.py tests/test_gpu_pipe.py tests/test_gpu_modules.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/wmt.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in scripts/bin/prev/libbessgpu.so bess_amd/libbessgpu.so; do
    timeout -k 10 300 python bench.py --lib $lib --only wm --no-cpu > /dev/null 2> $OUT/wmab.err || exit $?
    tail -1 $OUT/wmab.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'C4': d}))" >> $OUT/wm_pf_ab.jsonl
  done
done

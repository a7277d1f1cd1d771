#!/bin/bash
# round 4: ring ticket runs -- ring/pipe/plugin tests, stamps, C2 sweep (twice)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_pipe.py tests/test_bessd_wrappers.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t6.log 2>&1 || exit $?
timeout -k 10 240 python scripts/ring_trace.py 1 16 > $OUT/ring_trace6.jsonl 2> $OUT/ring_trace6.err || exit $?
for i in 1 2; do
  timeout -k 10 400 python bench.py --only sweep > $OUT/sweep_run_$i.json 2> $OUT/sweep_run.err || exit $?
done

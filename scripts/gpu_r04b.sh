#!/bin/bash
# round 4: ring tests, C5 probe calibration (rnd36s), ring ticket stamps, sweep
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_pipe.py tests/test_bessd_wrappers.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t4.log 2>&1 || exit $?
timeout -k 10 240 scripts/bin/hbm_probe 2 s > $OUT/probe_s4.jsonl || exit $?
timeout -k 10 240 python scripts/ring_trace.py 1 16 > $OUT/ring_trace4.jsonl 2> $OUT/ring_trace4.err || exit $?
timeout -k 10 300 python bench.py --only sweep > $OUT/sweep4.json 2> $OUT/sweep4.err || exit $?

#!/bin/bash
# round 4: ring relay mode -- ring/pipe/plugin tests, stamps, relay vs BAR
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_pipe.py tests/test_bessd_wrappers.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t5.log 2>&1 || exit $?
timeout -k 10 240 python scripts/ring_trace.py 1 16 > $OUT/ring_trace5.jsonl 2> $OUT/ring_trace5.err || exit $?
timeout -k 10 400 python scripts/ring_desc_ab.py > $OUT/ring_desc.jsonl 2> $OUT/ring_desc.err || exit $?

#!/bin/bash
# round 4: pipe ring staging, coherent vs uncached (A/B build), e2e_pipe leg
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for uc in 0 1 0 1; do
  BG_PIPE_UC=$uc timeout -k 10 300 python bench.py --lib scripts/bin/libbessgpu_ab.so --only pipe > $OUT/pipe_uc$uc.json 2>> $OUT/pipe_uc.err || exit $?
  tail -1 $OUT/pipe_uc.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'uc': $uc, 'em_ring': d['ExactMatch_64B']['Mpps_by_threads_ring_batch1024_depth8'], 'parity': d['ExactMatch_64B']['parity_ring_batch1024_depth8']}))" >> $OUT/pipe_uc.jsonl
done

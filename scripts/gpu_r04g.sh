#!/bin/bash
# round 4: e2e pipe leg, previous commit's library vs ticket runs, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for rep in 1 2; do
  for lib in scripts/bin/libbessgpu_prev.so bess_amd/libbessgpu.so; do
    timeout -k 10 300 python bench.py --lib $lib --only pipe > /dev/null 2> $OUT/pab.err || exit $?
    tail -1 $OUT/pab.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); e=d['ExactMatch_64B']; print(json.dumps({'lib': '$lib', 'ring': e['Mpps_by_threads_ring_batch1024_depth8'], 'l4096': e['Mpps_by_threads_launch_batch4096_depth4'], 'parity': e['parity_ring_batch1024_depth8']}))" >> $OUT/pipe_ab.jsonl
  done
done

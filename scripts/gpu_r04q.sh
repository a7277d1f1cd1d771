#!/bin/bash
# round 4: HashLB fields mode as a header-line op -- tests, then A/B (A/B
# build, BG_HLB_FIELDS_LANE=1: the lane-per-packet kernel), two reps
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_hashlb.py tests/test_hashlb.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t23.log 2>&1 || exit $?
for rep in 1 2; do
  for k in 1 0; do
    BG_HLB_FIELDS_LANE=$k timeout -k 10 300 python bench.py --lib scripts/bin/libbessgpu_ab.so --only hashlb --no-cpu > /dev/null 2> $OUT/hlb.err || exit $?
    tail -1 $OUT/hlb.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'lane': $k, 'fields': d.get('fields', d)}))" >> $OUT/hlb_ab.jsonl
  done
done

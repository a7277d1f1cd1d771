#!/bin/bash
# round 4: plugin pipes sized full slots first (A/B against the previous driver)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for rep in 1 2; do
  for d in scripts/bin/drive_prev tests/bessd_shell/build/drive; do
    timeout -k 10 600 python bench.py --drive $d --only plugin > /dev/null 2> $OUT/pk.err || exit $?
    tail -1 $OUT/pk.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'drive': '$d', 'plugin': d['Mpps_by_workers'], 'cpu': d['cpu_same_harness']['Mpps_by_workers'], 'parity': d['parity']}))" >> $OUT/plugin_ab.jsonl
    timeout -k 10 600 python bench.py --drive $d --only plugin_pool > /dev/null 2> $OUT/pk.err || exit $?
    tail -1 $OUT/pk.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'drive': '$d', 'pool_wm': d['WildcardMatch'], 'pool_l4': d['L4Checksum']}))" >> $OUT/plugin_ab.jsonl
  done
done

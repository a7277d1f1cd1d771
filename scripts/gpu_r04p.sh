#!/bin/bash
# round 4: the pipes' per-slot ring check without the module lock -- pipe
# tests, then the plugin leg against the previous library (LD_LIBRARY_PATH
# before the driver's RUNPATH), alternating
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipe.py tests/test_bessd_wrappers.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t19.log 2>&1 || exit $?
for rep in 1 2; do
  for L in prev new; do
    if [ $L = prev ]; then export LD_LIBRARY_PATH=$PWD/scripts/bin/prev; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 600 python bench.py --only plugin > /dev/null 2> $OUT/pq.err || exit $?
    tail -1 $OUT/pq.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$L', 'plugin': d['Mpps_by_workers'], 'cpu': d['cpu_same_harness']['Mpps_by_workers'], 'stats16': d['worker0_pipe_stats'].get('16','')[:160]}))" >> $OUT/plugin_lock_ab.jsonl
  done
done
unset LD_LIBRARY_PATH

#!/bin/bash
# HBM read calibration (scripts/hbm_probe.hip) + tests + bench on one box
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
run() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc" >> "$OUT/steps.log"; if [ $rc -gt 1 ]; then exit $rc; fi; }
hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_probe scripts/hbm_probe.hip > "$OUT/probe_build.log" 2>&1 || exit 3
run probe 300 /tmp/hbm_probe 1
run tests 900 python -m pytest tests -m gpu -q -rf --timeout 600
run bench 900 python bench.py ${BENCH_ARGS:-}

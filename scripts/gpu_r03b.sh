#!/bin/bash
# Round-3 measurement call: the ring's per-ticket trace (A/B build), the
# FETCH_SIZE / WRITE_SIZE passes of the run-time compiled C4 kernels (both
# layouts), the SQ counters of the C4 kernels. Each step under its own
# limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
for step in ${STEPS:-trace pmc sq}; do
  case $step in
    trace) timeout -k 10 240 python -u scripts/ring_trace.py 1 4 16 > $OUT/ring_trace.jsonl 2> $OUT/ring_trace.err ;;
    pmc)   PMC_WL="wm wm2k" timeout -k 10 700 bash scripts/gpu_full.sh pmc > $OUT/pmc.log 2>&1 ;;
    sq)    timeout -k 10 500 bash scripts/wm_pmc.sh > $OUT/wm_pmc.log 2>&1 ;;
  esac
  rc=$?; echo "$step rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

#!/bin/bash
# Measurement session (round 3): FETCH_SIZE calibration of the scattered
# shapes (gpu_calib.sh), SQ counters of the C4 kernels (wm_pmc.sh: the
# run-time compiled and the ahead-of-time kernel), C4 phase timing
# (variants.py wmphase, A/B build). Each step under its own limit; stops at
# the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for step in ${STEPS:-calib pmc phase}; do
  case $step in
    calib) timeout -k 10 600 bash scripts/gpu_calib.sh > $OUT/calib.log 2>&1 ;;
    pmc)   timeout -k 10 500 bash scripts/wm_pmc.sh > $OUT/wm_pmc.log 2>&1 ;;
    phase) timeout -k 10 300 python -u scripts/variants.py wmphase > $OUT/wmphase.json 2> $OUT/wmphase.err ;;
  esac
  rc=$?; echo "$step rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

#!/bin/bash
# Measurement session (round 3): the -m gpu suite, a same-box A/B of the C4
# kernels (product library vs the measurement build with software-pipelined
# checks, BG_WM_PIPE), C4 phase timing (variants.py wmphase), FETCH_SIZE
# calibration of the scattered shapes (gpu_calib.sh), SQ counters of the C4
# kernels (wm_pmc.sh). Each step under its own limit; stops at the first
# failure. STEPS selects steps.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for step in ${STEPS:-tests ab phase calib pmc}; do
  case $step in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
             --timeout-method thread > $OUT/tests.log 2>&1 ;;
    ab)    for rep in 1 2; do
             { [ ! -f bess_amd/libbessgpu_prev.so ] || timeout -k 10 180 python scripts/wm_ab.py bess_amd/libbessgpu_prev.so >> $OUT/ab.jsonl 2>> $OUT/ab.err; } &&
             timeout -k 10 180 python scripts/wm_ab.py >> $OUT/ab.jsonl 2>> $OUT/ab.err &&
             WM_AB_FLAGS=${WM_AB_FLAGS:-512} timeout -k 10 180 python scripts/wm_ab.py scripts/bin/libbessgpu_ab.so >> $OUT/ab.jsonl 2>> $OUT/ab.err || break
           done ;;
    calib) timeout -k 10 600 bash scripts/gpu_calib.sh > $OUT/calib.log 2>&1 ;;
    pmc)   timeout -k 10 500 bash scripts/wm_pmc.sh > $OUT/wm_pmc.log 2>&1 ;;
    phase) timeout -k 10 300 python -u scripts/variants.py wmphase > $OUT/wmphase.json 2> $OUT/wmphase.err ;;
  esac
  rc=$?; echo "$step rc=$rc"; tail -2 $OUT/tests.log 2>/dev/null | head -1; [ $rc -ne 0 ] && exit $rc
done
exit 0

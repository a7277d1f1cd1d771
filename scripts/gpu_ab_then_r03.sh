#!/bin/bash
# A/B of two library builds on scripts/wm_ab.py, then the round-3 session
# (scripts/gpu_r03.sh) with the product library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/ab_libs.sh scripts/wm_ab.py ab_libs/libbessgpu_base.so ab_libs/libbessgpu_new.so || exit $?
cat gpurun_out/ab.jsonl
bash scripts/gpu_r03.sh "$@"

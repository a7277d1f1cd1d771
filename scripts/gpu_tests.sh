#!/bin/bash
# GPU parity suite on one box: `gpurun -- bash scripts/gpu_tests.sh [pytest args]`
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log
exit $rc

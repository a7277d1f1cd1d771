#!/bin/bash
# round 4: pair loads on any stride -- WM tests, then C4 through the product library
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wm_jit.py tests/test_gpu_configs.py tests/test_gpu_pipe.py tests/test_gpu_parity.py tests/test_attr_fields.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t16.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --only wm > $OUT/wm16.json 2> $OUT/wm16.err || exit $?

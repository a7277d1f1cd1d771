#!/bin/bash
# Round 5: the streamed tag-word kernel with the software-pipelined consumer:
# parity, C4 times beside the unstreamed form, phases; ring stamps at
# 1024-packet tickets.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05f"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
  return 0
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_wm_jit.py "tests/test_gpu_configs.py::test_c4_imix_2k_slots" \
  "tests/test_gpu_configs.py::test_c4_header_slab_full_size" \
  "tests/test_gpu_parity.py::test_wm_vs_oracle" "tests/test_gpu_parity.py::test_wm_tags_fewer_direct_tuples" \
  "tests/test_gpu_parity.py::test_wm_direct_tuples_vs_oracle" "tests/test_gpu_parity.py::test_wm_priority_ties"
step wm 300 python -u bench.py --only wm --no-cpu --steps 20 --warmup 5
step wm2 300 python -u bench.py --only wm --no-cpu --steps 20 --warmup 5
step phase 600 python -u scripts/variants.py wmphase
step trace 300 python -u scripts/ring_trace.py --batch=1024 4 16
echo done >> "$OUT/steps.log"

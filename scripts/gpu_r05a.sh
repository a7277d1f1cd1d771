#!/bin/bash
# Round 5, first call: the new parity tests (P11 pipe/plugin staging,
# permuted attr offsets, 1500 B ExactMatch), then the 1500 B leg and the
# pooled plugin legs. Stops at the first step that ends in anything but
# success / test failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05a"
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
  tests/test_gpu_pipe.py tests/test_attr_fields.py \
  "tests/test_bessd_wrappers.py::test_l4_checksum_plugin_reads_past_data_len" \
  "tests/test_bessd_wrappers.py::test_deferred_pipeline_l4_checksum_and_acl" \
  "tests/test_gpu_configs.py::test_em_1500b_full_size" tests/test_rewrite.py tests/test_gpu_ring.py
step em1500 300 python -u bench.py --only em1500 --steps 20 --warmup 5
step pool 600 python -u bench.py --only plugin_pool
echo done >> "$OUT/steps.log"

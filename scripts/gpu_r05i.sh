#!/bin/bash
# Round 5: C3's checksum launch timed several ways in one process (the bench
# leg gave 0.339 ms where variants.py gave 0.298 on the same box)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05i"
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
step timing 300 python -u scripts/ck_timing.py
step c3 300 python -u bench.py --only cksum --no-cpu
step probe 300 ./scripts/bin/hbm_probe 2 c
step ck 600 python -u scripts/variants.py ck
for v in 0 8; do
  step pmc_f_$v 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f_$v" -o pmc -- python3 "$GRAFT_REPO_ROOT/scripts/ck_timing.py" ab=$v
  step pmc_w_$v 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w_$v" -o pmc -- python3 "$GRAFT_REPO_ROOT/scripts/ck_timing.py" ab=$v
done
echo done >> "$OUT/steps.log"

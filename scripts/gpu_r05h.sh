#!/bin/bash
# Round 5: checksum kernel variants (LDS stash of the header line) and C3's
# PMC traffic; C2 / C3 bench legs on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05h"
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
step ck 600 python -u scripts/variants.py ck
step c3 300 python -u bench.py --only cksum --no-cpu --steps 20 --warmup 5
step pmc_ck_1 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_ck_1" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" --only cksum --no-cpu --steps 3 --warmup 1
step pmc_ck_2 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_ck_2" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" --only cksum --no-cpu --steps 3 --warmup 1
echo done >> "$OUT/steps.log"

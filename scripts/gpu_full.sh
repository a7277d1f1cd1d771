#!/bin/bash
# Full GPU session: tests, smoke, bench, rocprofv3 kernel stats + PMC passes.
# Stops at the first step that ends in anything but success / test failure.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/${OUTDIR:-.}"
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
MODE=${1:-all}
if [[ "$MODE" == *tests* ]] || [ "$MODE" = all ]; then
  step tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ "$MODE" == *bench* ]] || [ "$MODE" = all ]; then
  step bench 900 python bench.py
fi
if [[ "$MODE" == *prof* ]] || [ "$MODE" = all ]; then
  # kernel trace of the default bench command (every kernel of the line)
  # (the host end-to-end legs launch from 16 threads, which crashes the
  # tracer; every device-resident kernel of the line is traced)
  step prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-e2e
fi
if [[ "$MODE" == *pmc* ]] || [ "$MODE" = all ]; then
  rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
  i=0
  for C in ${PMC_SETS:-"FETCH_SIZE" "WRITE_SIZE"}; do
    i=$((i+1))
    for W in ${PMC_WL:-em cksum wm wm2k em1500 c5 hashlb acl iplookup ttl nat dnat rewrite}; do
      case $W in
        em) ARGS="--no-extra --no-cpu --steps 3 --warmup 1" ;;
        wm) ARGS="--only wm --wm-layout slab --no-cpu --steps 3 --warmup 1" ;;
        wm2k) ARGS="--only wm --wm-layout 2k --no-cpu --steps 3 --warmup 1" ;;
        dnat) ARGS="--only dnat --no-churn --no-cpu --steps 3 --warmup 1" ;;
        *) ARGS="--only $W --no-cpu --steps 3 --warmup 1" ;;
      esac
      step pmc_${W}_$i 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${W}_$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS
    done
  done
  python3 scripts/pmc_traffic.py "$OUT" "$OUT/traffic.json" > "$OUT/pmc_traffic.out" 2>&1 || true
fi
echo done >> "$OUT/steps.log"

#!/bin/bash
# Round 5: what bounds C4's header phase -- SQ / TA / TD / TCP counter passes
# on the WildcardMatch slab leg and, for comparison, C2's ExactMatch kernel
# (same 64 B slab shape); one rocprofv3 run per pass
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r05k"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# the slab shape with gates stored per tile vs gathered per 8-tile run
timeout -k 10 300 $R/scripts/bin/hbm_probe 1 c > "$OUT/probe_c.jsonl" 2> "$OUT/probe_c.err"
echo "== probe rc=$?" >> "$OUT/steps.log"
P1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
P3="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM"
for W in wm em; do
  case $W in
    wm) ARGS="--only wm --wm-layout slab --no-cpu --steps 3 --warmup 1" ;;
    em) ARGS="--no-extra --no-e2e --no-cpu --steps 3 --warmup 1" ;;
  esac
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    echo "== ${W}_$i" >> "$OUT/steps.log"
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_${W}_$i -o pmc -- python3 $R/bench.py $ARGS > "$OUT/${W}_$i.log" 2>&1
    rc=$?
    echo "== ${W}_$i rc=$rc" >> "$OUT/steps.log"
    if [ $rc -ne 0 ]; then echo "stopping" >> "$OUT/steps.log"; exit $rc; fi
    python3 $R/scripts/pmc_summary.py /tmp/pmc_${W}_$i > "$OUT/${W}_$i.json" 2>> "$OUT/steps.log"
    rm -rf /tmp/pmc_${W}_$i
  done
done
echo done >> "$OUT/steps.log"

#!/bin/bash
# Round 6 counter passes: `gpurun -- bash scripts/gpu_r06_pmc.sh OUTDIR [what]`
#   what: scatter (scripts/scatter_probe.hip variants) and/or placement
#   (scripts/slab_placement.py pmc), tcc (per-channel L2 requests of the
#   same run), mem (the L2's memory-side queue and DRAM credit stalls on
#   the scatter shapes and two streaming shapes), comma list; one rocprofv3
#   run per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
OUT="$R/gpurun_out/$1"
WHAT=${2:-scatter,placement}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
pass() {  # name cmd...
  local name=$1; shift
  local i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    echo "== ${name}_$i" >> "$OUT/steps.log"
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_${name}_$i -o pmc -- "$@" > "$OUT/${name}_$i.log" 2>&1
    rc=$?
    echo "== ${name}_$i rc=$rc" >> "$OUT/steps.log"
    if [ $rc -ne 0 ]; then echo "stopping" >> "$OUT/steps.log"; exit $rc; fi
    mkdir -p "$OUT/csv_${name}_$i"
    find /tmp/pmc_${name}_$i -name '*counter_collection.csv' -exec cp {} "$OUT/csv_${name}_$i/" \;
    rm -rf /tmp/pmc_${name}_$i
  done
}
if [[ ",$WHAT," == *",scatter,"* ]]; then
  for V in "vec2 512 1" "pair 512 1" "pair 256 4" "pairU4 256 1" "quad64 512 1"; do
    set -- $V
    pass "sc_$1_$2_$3" $R/scripts/bin/scatter_probe 16 $1 $2 $3 20
  done
fi
if [[ ",$WHAT," == *",placement,"* ]]; then
  pass placement python3 $R/scripts/slab_placement.py "$OUT/placement_pmc.json" pmc
fi
if [[ ",$WHAT," == *",tcc,"* ]]; then  # per-instance L2 channel requests, A vs the rest
  P1="TCC_EA0_RDREQ"; P2="TCC_REQ"
  pass placement_tcc python3 $R/scripts/slab_placement.py "$OUT/placement_tcc.json" pmc
fi
if [[ ",$WHAT," == *",mem,"* ]]; then  # the memory side: EA read queue and DRAM credit stalls
  P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
  P2="TCC_TAG_STALL_sum TCC_REQ_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  for V in "vec2 512 1" "pair 512 1" "quad64 512 1"; do
    set -- $V
    pass "mem_$1_$2_$3" $R/scripts/bin/scatter_probe 16 $1 $2 $3 20
  done
  pass mem_full16 $R/scripts/bin/hbm_probe 16 only full16 2 20
  pass mem_slab66 $R/scripts/bin/hbm_probe 16 only slab66 2 20
fi
echo done >> "$OUT/steps.log"

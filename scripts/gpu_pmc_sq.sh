#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 --pmc run per pass) on chosen
# bench workloads: where a latency-bound kernel's wave cycles go.
#   WL="wm c5" scripts/gpu_pmc_sq.sh
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum"
for W in ${WL:-wm}; do
  if [ $W = em ]; then ARGS="--no-extra --no-cpu --steps 3 --warmup 1"; elif [ $W = wm ]; then ARGS="--only wm --wm-layout slab --no-cpu --steps 3 --warmup 1"; else ARGS="--only $W --no-cpu --steps 3 --warmup 1"; fi
  i=0
  for C in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_${W}_$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/sq_${W}_$i.out" 2>&1
    rc=$?; echo "sq_${W}_$i rc=$rc" >> "$OUT/steps.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done

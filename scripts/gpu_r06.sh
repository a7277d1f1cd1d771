#!/bin/bash
# Round-6 GPU call: `gpurun -- bash scripts/gpu_r06.sh OUTDIR [steps]`
# steps (comma list): wide (the full-width WildcardMatch tests), tests (the
# whole -m gpu suite), smoke, bench (default bench line), prof (kernel
# trace of the bench per leg). Stops at the first step that ends in
# anything but success / test failure. sel: the tests named in $SEL;
# prof: scripts/prof_legs.py over $LEGS (default: every leg).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"
STEPS=${2:-wide,tests,smoke}
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
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has wide; then
  step wide 600 python -u -m pytest tests/test_gpu_wm_wide.py -m gpu -v -rf --timeout 300 --timeout-method thread
fi
if has sel; then  # SEL: test files / node ids
  step sel 600 python -u -m pytest $SEL -m gpu -v -rf --timeout 300 --timeout-method thread
fi
if has tests; then
  step tests 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
fi
if has smoke; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has prof; then  # a kernel trace per bench leg (scripts/prof_legs.py)
  step prof 1000 python scripts/prof_legs.py run "$OUT/legs" $LEGS
  python scripts/prof_legs.py summary "$OUT/legs" > "$OUT/kernels_by_leg.md" 2>&1 || true
fi
if has sweep; then  # the C2 batch sweep alone (ring rows)
  step sweep 600 python bench.py --only sweep --no-cpu
fi
if has placement; then  # C4's 2 KB-slot time over separately placed slabs
  step placement 600 python scripts/slab_placement.py "$OUT/placement.json" $PLACEMENT
fi
if has ringab; then  # the sweep's ring rows: product vs $RINGLIBS, interleaved
  for rep in 1 2; do
    for L in product $RINGLIBS; do
      if [ "$L" = product ]; then LA=""; else LA="--lib scripts/bin/libbessgpu_$L.so"; fi
      step "sweep_${L}_$rep" 600 python bench.py --only sweep --no-cpu $LA
      if [ -n "$PIPEAB" ]; then
        step "pipe_${L}_$rep" 600 python bench.py --only pipe --no-cpu $LA
      fi
    done
  done
fi
if has c2ab; then  # the headline kernel: product vs $C2LIBS, interleaved
  for rep in 1 2; do
    for L in product $C2LIBS; do
      if [ "$L" = product ]; then LA=""; else LA="--lib scripts/bin/libbessgpu_$L.so"; fi
      step "c2_${L}_$rep" 300 python bench.py --no-extra --no-cpu --steps 200 --warmup 20 $LA
      if [ -n "$C5AB" ]; then
        step "c5_${L}_$rep" 300 python bench.py --only c5 --no-cpu $LA
      fi
    done
  done
fi
if has legab; then  # bench legs $ABLEGS: product vs $LEGLIBS, interleaved ($REPS times)
  for rep in $(seq 1 ${REPS:-2}); do
    for L in product $LEGLIBS; do
      if [ "$L" = product ]; then LA=""; else LA="--lib scripts/bin/libbessgpu_$L.so"; fi
      for W in $ABLEGS; do
        step "leg_${W}_${L}_$rep" 300 python bench.py --only $W --no-cpu $LA
      done
    done
  done
fi
if has gate; then  # scripts/gate_probe.hip: C2's shape, gate stores placed differently
  step gate 300 scripts/bin/gate_probe 1
fi
if has scatter; then  # scripts/scatter_probe.hip, every variant
  step scatter 600 scripts/bin/scatter_probe 16
fi
if has legs; then  # bench legs alone: $ONLY (e.g. "wm em1500")
  for W in $ONLY; do
    step "leg_$W" 600 python bench.py --only $W --no-cpu
  done
fi
if has dip; then  # the ring sweep's rows, every repetition (scripts/ring_dip_probe.py)
  step dip 600 python scripts/ring_dip_probe.py "$OUT/dip.json" 8
fi
if has bench; then
  step bench 900 python3 bench.py --gpus 1 --steps 20 --warmup 5
fi
echo done >> "$OUT/steps.log"

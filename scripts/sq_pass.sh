#!/bin/bash
# One rocprofv3 --pmc pass (counters in $P) over a bench workload ($W),
# summarised per kernel on the box (scripts/pmc_summary.py).
#   P="SQ_WAVE_CYCLES SQ_WAIT_ANY" W=dnat bash scripts/sq_pass.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
if [ "$W" = wm ]; then ARGS="--only wm --wm-layout slab --no-cpu --steps 3 --warmup 1"; else ARGS="--only $W --no-cpu --steps 3 --warmup 1"; fi
timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d /tmp/sqp -o pmc -- python3 $R/bench.py $ARGS > $O/sq_pass_$W.log 2>&1 || exit 1
python3 $R/scripts/pmc_summary.py /tmp/sqp > $O/sq_pass_$W.json

#!/bin/bash
# Measured ceilings and FETCH_SIZE calibration for the scattered access
# shapes: scripts/hbm_probe.hip timed (s: 2 KB-stride
# header reads, the C5 random-probe shape; r: streaming reference shapes),
# then one rocprofv3 --pmc pass per (shape, counter set), 10 launches each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/calib
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -o /tmp/hbm_probe $R/scripts/hbm_probe.hip > $O/build.log 2>&1 || exit 3
timeout -k 10 240 /tmp/hbm_probe 2 s > $O/probe_s.jsonl || exit 4
timeout -k 10 240 /tmp/hbm_probe 2 > $O/probe_r.jsonl || exit 4
for shape in full16 em32 s2k32 s2k64 rnd36; do
  i=0
  for P in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $P -d /tmp/cal_${shape}_$i -o run --output-format csv \
        -- /tmp/hbm_probe 2 only $shape 2 10 > $O/${shape}_$i.log 2>&1 \
      || { echo "pass $shape $i failed rc=$?" >> $O/status; continue; }
    python3 $R/scripts/pmc_summary.py /tmp/cal_${shape}_$i > $O/${shape}_$i.json 2>> $O/status
    rm -rf /tmp/cal_${shape}_$i
    echo "pass $shape $i ok" >> $O/status
  done
done
cat $O/probe_s.jsonl

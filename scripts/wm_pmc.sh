#!/bin/bash
# SQ counter passes over scripts/wm_ab.py (C4), one rocprofv3 run per pass;
# keeps only a per-kernel summary (the raw per-dispatch CSVs are large)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wm_pmc
mkdir -p $O
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d /tmp/pmc$i -o run --output-format csv -- python3 $R/scripts/wm_ab.py > $O/p$i.log 2>&1 || { echo "pass $i failed" >> $O/status; exit 1; }
  python3 $R/scripts/pmc_summary.py /tmp/pmc$i > $O/p$i.json 2>> $O/status || { echo "summary $i failed" >> $O/status; exit 1; }
  rm -rf /tmp/pmc$i
  echo "pass $i ok" >> $O/status
done

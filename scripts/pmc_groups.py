#!/usr/bin/env python3
"""Counter passes of scripts/gpu_r06_pmc.sh, per dispatch group, with the
derived request figures of DESIGN §3 (L2 requests in flight per CU).

    python scripts/pmc_groups.py OUTDIR [> profiles/r06/pmc_groups.json]

For every csv_<name>_<pass>/ directory: the dispatches of the kernel that
ran most often, in order; a `sc_*` run (scatter_probe: 1 + 20 launches of
one variant) is one group without its first dispatch; `placement` (
slab_placement.py pmc: 21 launches per slab, slabs in the order its JSON
lists them) is split into groups of 21, each without its first launch.
Derived, per group and launch:
  req_per_slot       TCP_TCC_READ_REQ / slots (L1 -> L2 read requests)
  latency_cycles     TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ
  inflight_per_cu    TCP_TCC_READ_REQ_LATENCY / (GRBM_GUI_ACTIVE / 8 XCDs)
                     / CUs: the read requests a CU's L1 has outstanding on
                     average (Little's law)
  ea_rd_inflight_chip  TCC_EA0_RDREQ_LEVEL / cycles: the L2s' read requests
                     outstanding to memory, chip-wide
  dram_credit_stall_per_cycle  TCC_EA0_RDREQ_DRAM_CREDIT_STALL / cycles (the
                     L2 channels waiting for DRAM credits, summed)
  utcl1_miss_per_slot  TCP_UTCL1_TRANSLATION_MISS / slots
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

CUS = 256
XCDS = 8


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "*.csv")):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> sum
    name, grid = {}, {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        name[k] = r["Kernel_Name"]
        grid[k] = int(r["Grid_Size"])
    return per, name


def main():
    out_dir = sys.argv[1]
    res = {}
    for d in sorted(glob.glob(os.path.join(out_dir, "csv_*_[0-9]"))):
        tag = os.path.basename(d)[4:]
        per, name = load(d)
        if not per:
            continue
        counts = defaultdict(int)
        for k in per:
            counts[name[k]] += 1
        main_k = max(counts, key=counts.get)
        ids = sorted(k for k in per if name[k] == main_k)
        if not tag.startswith("placement"):
            groups = [("all", ids[1:])]
            # 16 GiB of 2 KiB slots (scatter_probe), of 64 B slots (hbm_probe)
            slots = (256 << 20) if tag.startswith(("mem_full16", "mem_slab66")) else (8 << 20)
        else:
            groups = [("slab%d" % (i // 21), ids[i + 1:i + 21]) for i in range(0, len(ids), 21)]
            slots = 8 << 20
        base, pas = tag.rsplit("_", 1)
        for gname, g in groups:
            if not g:
                continue
            agg = defaultdict(float)
            for k in g:
                for c, v in per[k].items():
                    agg[c] += v / len(g)
            e = res.setdefault(base, {}).setdefault(gname, {})
            e.update({c: round(v, 1) for c, v in agg.items()})
            e["kernel"] = re.sub(r"\(.*", "", main_k)[:80]
            e["dispatches"] = len(g)
            req = e.get("TCP_TCC_READ_REQ_sum")
            lat = e.get("TCP_TCC_READ_REQ_LATENCY_sum")
            act = e.get("GRBM_GUI_ACTIVE")
            if req:
                e["req_per_slot"] = round(req / slots, 3)
                if lat:
                    e["latency_cycles"] = round(lat / req, 1)
            # GRBM_GUI_ACTIVE counts every XCD's busy cycles (8 per cycle)
            if lat and act:
                e["inflight_per_cu"] = round(lat / (act / XCDS) / CUS, 1)
            lev, ea = e.get("TCC_EA0_RDREQ_LEVEL_sum"), e.get("TCC_EA0_RDREQ_sum")
            if lev and act:
                e["ea_rd_inflight_chip"] = round(lev / (act / XCDS), 1)
                if ea:
                    e["ea_rd_latency_cycles"] = round(lev / ea, 1)
            st = e.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum")
            if st is not None and act:
                e["dram_credit_stall_per_cycle"] = round(st / (act / XCDS), 2)
            if e.get("TCP_UTCL1_TRANSLATION_MISS_sum") is not None:
                e["utcl1_miss_per_slot"] = round(e["TCP_UTCL1_TRANSLATION_MISS_sum"] / slots, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

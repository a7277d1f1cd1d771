#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (scripts/gpu_full.sh).

    python scripts/pmc_traffic.py gpurun_out profiles/r01_traffic.json

Reads every counter_collection.csv under gpurun_out/pmc_<workload>_<i>/,
averages each counter over the dispatches of the workload's kernel and
applies MI355X_MICROARCH.md's gfx950 corrections, calibrated per access
shape on known byte counts (profiles/r03_calibration.json):
  * FETCH_SIZE (KB) = TCC_EA0_RDREQ x 64 B. Wide streaming reads and dense
    slots make 128 B requests: x2 (the guide's correction). A 32 B window
    per 2 KB slot (C4 on 2 KB slots) makes one 64 B request: x1 (FETCH).
  * WRITE_SIZE (KB) is exact for 16 B/lane stores.
traffic = FETCH[wl] * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 bytes per launch.
Random table reads that hit the Infinity Cache are counted too (C5).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench workload -> substring of its timed kernel's name
KERNELS = {"em": "em_slab_kernel", "cksum": "cksum_kernel",
           "wm": "bg_wm_jit", "wm2k": "bg_wm_jit",  # the run-time compiled kernel
           "c5": "em_slab_kernel",
           "hashlb": "HlbOp<2>", "acl": "AclTreeOp", "iplookup": "Lpm16LdsOp",
           "ttl": "TtlOp<4>", "nat": "NatOp", "dnat": "dnat_fused_slab_kernel",
           "rewrite": "rewrite_kernel", "em1500": "em_pair_kernel"}
# algorithmic bytes per launch of each bench workload
ALGO = {"em": 66 * (16 << 20), "cksum": 1502 * (1 << 20),
        "wm": 66 * (8 << 20), "wm2k": 66 * (8 << 20), "c5": 66 * (16 << 20),
        "hashlb": 66 * (16 << 20), "acl": 66 * (16 << 20),
        "iplookup": 66 * (16 << 20), "ttl": 130 * (16 << 20),
        # StaticNAT writes back only the translated half (round 6): 66 + 64 / 2
        "nat": 98 * (16 << 20), "dnat": 130 * (16 << 20),
        "rewrite": 70 * (16 << 20), "em1500": 66 * (4 << 20)}
# FETCH_SIZE -> bytes factor by access shape (r03_calibration.json)
FETCH = {"wm2k": 1, "em1500": 1}


def collect(root, wl):
    vals = defaultdict(list)
    for p in glob.glob(os.path.join(root, "pmc_%s_*" % wl, "**", "*counter_collection.csv"),
                       recursive=True):
        per = defaultdict(float)  # (dispatch, counter) -> value
        with open(p) as f:
            for r in csv.DictReader(f):
                if KERNELS[wl] not in r["Kernel_Name"]:
                    continue
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in per.items():
            vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items() if v}


def main():
    root, out = sys.argv[1], sys.argv[2]
    res = {}
    for wl in KERNELS:
        c = collect(root, wl)
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = FETCH.get(wl, 2) * c["FETCH_SIZE"] * 1024
        write = c["WRITE_SIZE"] * 1024
        e = {"traffic_bytes": round(fetch + write),
             "fetch_bytes_corrected": round(fetch),
             "write_bytes": round(write),
             "algorithmic_bytes": ALGO[wl],
             "fetch_factor": FETCH.get(wl, 2),
             "traffic_over_algorithmic": round((fetch + write) / ALGO[wl], 4),
             "raw": {k: round(v, 1) for k, v in c.items()}}
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            e["l2_hit_rate"] = round(c["TCC_HIT_sum"] /
                                     max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        res[wl] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

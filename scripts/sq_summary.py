#!/usr/bin/env python3
"""Average SQ/TCC counters per dispatch of a workload's kernel from
scripts/gpu_pmc_sq.sh output:  python scripts/sq_summary.py gpurun_out wm"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(__file__))
from pmc_traffic import KERNELS  # noqa: E402


def main():
    root, wl = sys.argv[1], sys.argv[2]
    per = defaultdict(float)
    disp = defaultdict(set)
    for p in glob.glob(os.path.join(root, "sq_%s_*" % wl, "**", "*counter_collection.csv"),
                       recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if KERNELS[wl] not in r["Kernel_Name"]:
                    continue
                per[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((p, r["Dispatch_Id"]))
    c = {k: v / len(disp[k]) for k, v in per.items()}
    for k in sorted(c):
        print("%-24s %14.0f" % (k, c[k]))
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if k in c:
                print("%-24s %6.1f %% of wave cycles" % (k, 100 * c[k] / w))
    if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
        print("VALU insts per wave      %.0f" % (c["SQ_INSTS_VALU"] / c["SQ_WAVES"]))
    if "TCC_HIT_sum" in c:
        print("L2 hit rate              %.3f" % (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))


if __name__ == "__main__":
    main()

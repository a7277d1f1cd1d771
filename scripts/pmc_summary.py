#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc output directory (argv[1]): per kernel name,
the mean of each counter over its dispatches, split into dispatch halves
(first / second half of that kernel's dispatches, e.g. two layouts timed one
after the other). Prints JSON."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    files = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter
    for r in rows:
        k = r.get("Kernel_Name", "?")[:90]
        d = int(r.get("Dispatch_Id", 0))
        per[k][d][r["Counter_Name"]] = per[k][d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {}
    for k, ds in per.items():
        ids = sorted(ds)
        halves = [ids[:len(ids) // 2], ids[len(ids) // 2:]] if len(ids) > 1 else [ids]
        out[k] = []
        for h in halves:
            agg = defaultdict(float)
            for d in h:
                for c, v in ds[d].items():
                    agg[c] += v / len(h)
            out[k].append({"dispatches": len(h), **{c: round(v, 1) for c, v in agg.items()}})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The ring rows of interleaved sweep runs (scripts/gpu_r06.sh ringab) in one
JSON: python scripts/collect_ringab.py OUTDIR > profiles/r06/ring_ab_<call>.json"""
import glob
import json
import os
import sys

res = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "sweep_*.err"))):
    name = os.path.basename(f)[len("sweep_"):-len(".err")]
    for ln in open(f):
        if ln.startswith("{"):
            d = json.loads(ln)
            res[name] = {k: d[k] for k in ("persistent", "persistent_4sub", "persistent_16sub")
                         if k in d}
print(json.dumps({"what": "C2 ring sweep rows (Mpps by packets per ticket), each library "
                          "twice, interleaved, one box (bench.py --only sweep [--lib])",
                  "runs": res}, indent=1))

#!/usr/bin/env python3
"""The headline (C2) and C5 legs of interleaved library runs
(scripts/gpu_r06.sh c2ab) in one JSON:
python scripts/collect_c2ab.py OUTDIR > profiles/r06/c2_ab_<call>.json"""
import glob
import json
import os
import sys

res = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "c[25]_*.out")) +
                glob.glob(os.path.join(sys.argv[1], "c5_*.err"))):
    name = os.path.basename(f).rsplit(".", 1)[0]
    lines = [ln for ln in open(f) if ln.startswith("{")]
    if not lines:
        continue
    d = json.loads(lines[-1])
    if name.startswith("c2_"):
        res[name] = {"kernel_ms": d["roofline"]["kernel_ms"], "frac": d["roofline"]["frac"],
                     "ms_per_step": d["ms_per_step"], "parity": d["parity"]}
    else:
        res[name] = {"ms_per_step": d.get("ms_per_step"), "parity": d.get("parity"),
                     "frac": (d.get("roofline") or {}).get("frac")}
print(json.dumps({"what": "C2 (bench.py --no-extra --steps 200) and C5 (--only c5) per "
                          "library build, each twice, interleaved, one box", "runs": res},
                 indent=1))

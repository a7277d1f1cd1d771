#!/usr/bin/env python3
"""C2's kernel launch by launch after the slab arrives (the driver's --steps
20 --warmup 5 read 3-7 % slower than 200 steps): each launch timed with its
own HIP events, 300 launches, for a slab that is
  h2d      just uploaded from the host (the bench's case),
  h2d_idle uploaded, then 200 ms of host idle,
  devread  uploaded, then read once on the device (a sum over it),
  devcopy  uploaded, then rewritten by a device copy (slab -> new slab),
  fresh    a new allocation filled by a device kernel (never crossed PCIe).
Each case has its own allocation; the order is interleaved twice.
Usage: python scripts/first_launch_probe.py OUT.json [settle]
(settle: one slab, each kind of untimed settle work before the launches)"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def main():
    out = sys.argv[1]
    dev = torch.device("cuda:0")
    n = 16 << 20
    keys, gates, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=0x5EED)
    host = torch.from_numpy(frames.reshape(-1))
    del frames
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    t.sync(0)
    d_gates = torch.empty(n, dtype=torch.int16, device=dev)
    ref = None
    res = {"what": __doc__.split("\n")[0], "cases": []}

    def run(d, name, rep):
        nonlocal ref
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(300)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record()
            t.classify(d, 64, n, 8192, d_gates)
            b.record()
        torch.cuda.synchronize()
        ms = [round(a.elapsed_time(b), 4) for a, b in ev]
        g = d_gates[:1 << 20].cpu()
        if ref is None:
            ref = g
        ok = bool(torch.equal(g, ref))
        r = {"case": name, "rep": rep, "first5": ms[:5], "first25_avg": round(float(np.mean(ms[:25])), 4),
             "launch5_25_avg": round(float(np.mean(ms[5:25])), 4),
             "last100_avg": round(float(np.mean(ms[-100:])), 4),
             "by25": [round(float(np.mean(ms[i:i + 25])), 4) for i in range(0, 300, 25)],
             "same_gates": ok}
        print(json.dumps(r), flush=True)
        res["cases"].append(r)

    if len(sys.argv) > 2 and sys.argv[2] == "settle":
        # the slab kept; 300 ms of host idle, then ~100 ms of untimed device
        # work of each kind before the 300 launches: none, bench.py's
        # multiply over 64 MB (it stays in the 256 MB Infinity Cache), the
        # same over 1 GB (through HBM), the headline's own launch
        d = host.to(dev)
        x64 = torch.ones(16 << 20, dtype=torch.float32, device=dev)
        x1g = torch.ones(256 << 20, dtype=torch.float32, device=dev)
        works = {"none": None, "mul64m": lambda: x64.mul_(1.0),
                 "mul1g": lambda: x1g.mul_(1.0),
                 "own": lambda: t.classify(d, 64, n, 8192, d_gates)}
        for rep in (1, 2):
            for name, fn in works.items():
                torch.cuda.synchronize()
                time.sleep(0.3)
                if fn is not None:
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < 0.1:
                        for _ in range(8):
                            fn()
                        torch.cuda.synchronize()
                run(d, "settle_" + name, rep)
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
        return
    for rep in (1, 2):
        for name in ("h2d", "h2d_idle", "devread", "devcopy", "fresh"):
            if name == "fresh":
                src = host.to(dev)
                d = torch.empty_like(src)
                d.copy_(src)
                del src
            else:
                d = host.to(dev)
            torch.cuda.synchronize()
            if name == "h2d_idle":
                time.sleep(0.2)
            elif name == "devread":
                _ = d.view(torch.int32).sum().item()
            elif name == "devcopy":
                d2 = torch.empty_like(d)
                d2.copy_(d)
                del d
                d = d2
            run(d, name, rep)
            del d
            torch.cuda.empty_cache()
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

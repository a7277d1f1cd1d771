#!/usr/bin/env python3
"""C4 floor probe: on the C4 slab (8M IMIX frames in 2 KB slots, the 1M
generated frames repeated 8x), time (a) the WildcardMatch kernel with 1, 2,
4 and 8 tuples of the same rule set, (b) ExactMatch (1K rules, LDS table):
the header-line read cost at this stride with almost no table work."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    n0, rep = 1 << 20, 8
    n = n0 * rep
    rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n0, stride=2048)
    d = torch.from_numpy(frames.reshape(-1)).to(dev).repeat(rep)
    dg = torch.empty(n, dtype=torch.int16, device=dev)
    out = {}
    masks = [m.tobytes() for m in rm]
    order = list(dict.fromkeys(masks))
    for nt in (1, 2, 4, 8):
        t = F.WmTable(P.FIVE_TUPLE)
        keep = set(order[:nt])
        for k, m, p, g in zip(rk, rm, prio, gates):
            if m.tobytes() in keep:
                t.add(k.tobytes(), m.tobytes(), int(p), int(g))
        out["wm_%d_tuples_ms" % nt] = round(timed(lambda: t.classify(d, 2048, n, 8192, dg)), 4)
        out["wm_%d_tuples_table" % nt] = t.table_info()
    keys, egates, _ = P.em_workload(1000, 1024, seed=1)
    e = F.EmTable(P.em_fields_5tuple())
    e.add_many(keys, egates)
    out["em_1k_ms"] = round(timed(lambda: e.classify(d, 2048, n, 8192, dg)), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

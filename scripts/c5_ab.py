#!/usr/bin/env python3
"""ExactMatch over 16 M resident 64 B packets -- C5 (1 M rules, table in
HBM/MALL) or, with argv[2] = 1000, C2 (table in LDS) -- timed through a
given build of libbessgpu.so (argv[1]; default the product library). Run once per library in separate processes on one box to compare
kernel versions. Prints one JSON line with a checksum of the gates."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def main():
    n, nr = 16 << 20, int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    keys, gates, frames = P.em_workload(nr, n, seed=0xC5, pkt_seed=0xC55)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    del frames
    g = torch.empty(n, dtype=torch.int16, device="cuda")
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    t.sync(0)
    t.classify(d, 64, n, 8192, g)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            t.classify(d, 64, n, 8192, g)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20)
    got = g.cpu().numpy().view(np.uint16)
    crc = int(np.bitwise_xor.reduce(got.astype(np.uint64) *
                                     np.arange(1, n + 1, dtype=np.uint64)))
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "rules": nr, "ms": round(best, 4),
                      "frac": round(66 * n / (best * 1e-3) / 8e12, 4), "gates_crc": crc}))


if __name__ == "__main__":
    main()

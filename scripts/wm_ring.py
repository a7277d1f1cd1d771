#!/usr/bin/env python3
"""The persistent ring over a WildcardMatch table (bg_wm_ring_create): C4's
100 K rules over 8 masks, 1 M IMIX header lines in a dense 64 B slab on the
device, one submitter, tickets of B packets; Mpps per B and the gates
against the launched kernel's. With the A/B build (argv[1]) and BG_RING_TRACE
the per-ticket stamps too. One JSON line per B."""
import json
import os
import sys
import time

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
    n = 1 << 20
    rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    h = torch.from_numpy(np.ascontiguousarray(frames[:, :64]).reshape(-1)).cuda()
    ref = torch.empty(n, dtype=torch.int16, device="cuda")
    t.classify(h, 64, n, 8192, ref)
    torch.cuda.synchronize()
    want = ref.cpu().numpy()
    g = torch.empty(n, dtype=torch.int16, device="cuda")
    for blocks in (0, 512):
        ring = F.Ring(t, slots=4096, blocks=blocks)
        ring.set_coherence(0, 0)
        for B in (32, 256, 1024, 4096, 65536):
            g.fill_(-1)
            ring.run(h, 64, n, B, 8192, g)  # warm
            t0 = time.perf_counter()
            ring.run(h, 64, n, B, 8192, g)
            dt = time.perf_counter() - t0
            ok = bool((g.cpu().numpy() == want).all())
            print(json.dumps({"blocks": blocks or "4/CU", "batch": B,
                              "Mpps": round(n / dt / 1e6, 1), "same_gates": ok}), flush=True)
        ring.close()


if __name__ == "__main__":
    main()

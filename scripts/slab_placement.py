#!/usr/bin/env python3
"""Does C4's 2 KB-slot time depend on where its 16 GB slab lies? (DESIGN §8
open item 7)

    python scripts/slab_placement.py OUT.json [pmc]

(pmc: 21 launches per slab and no settle, for rocprofv3 --pmc passes whose
per-dispatch rows are then grouped by slab in this order; many: the bench's
allocation, then six hipDeviceMallocContiguous and six plain 16 GB
allocations, interleaved and all kept.)

One process: the C4 rule set (100 K WildcardMatch rules over 8 masks) and
8 M IMIX frames in 2 KB slots, timed (the run-time compiled kernel, 100
launches after a settle, HIP events) over
  * slab A: the bench's allocation (torch.repeat of the 1 M frames, 16 GB);
  * D1-3 / E1-3: hipExtMallocWithFlags with hipDeviceMallocContiguous / 0,
    interleaved;
  * slab B: a second torch allocation holding the same bytes;
  * slab A again (the first measurement's repeatability);
  * A2: a torch allocation made after A was freed;
  * slab C: one 16 GB + 4 KB allocation, the frames copied to byte offsets
    0 and 1024 inside it (the windows' address bits below and at the slot
    size move; the physical pages do not).
Each entry records the slab's device address modulo 2 MB and 1 GB."""
import json
import os
import sys
import time

import ctypes as C

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


class Raw:
    """a device address where the bess_amd wrappers take a tensor"""
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


def main():
    out_path = sys.argv[1]
    n0, rep = 1 << 20, 8
    n = n0 * rep
    rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n0, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    t.jit_wait()
    dg = torch.empty(n, dtype=torch.int16, device="cuda")
    ref = None

    pmc = len(sys.argv) > 2 and sys.argv[2] == "pmc"

    def timed(slab, k=100):
        t.classify(slab, 2048, n, 8192, dg)
        torch.cuda.synchronize()
        if pmc:  # counter passes: 1 + 20 launches per slab, nothing else
            k = 20
        t0 = time.perf_counter()
        while not pmc and time.perf_counter() - t0 < 0.1:  # settle (as bench.py clock_settle)
            for _ in range(8):
                t.classify(slab, 2048, n, 8192, dg)
            torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(k):
            t.classify(slab, 2048, n, 8192, dg)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / k

    def entry(name, slab):
        nonlocal ref
        ms = timed(slab)
        g = dg.cpu().numpy()
        if ref is None:
            ref = g.copy()
        p = slab.data_ptr()
        e = {"slab": name, "ms": round(ms, 4), "addr_mod_2MB": p % (2 << 20),
             "addr_mod_1GB": p % (1 << 30), "same_gates": bool((g == ref).all())}
        print(json.dumps(e), flush=True)
        return e

    res = []
    if len(sys.argv) > 2 and sys.argv[2] == "many":
        # six physically contiguous and six plain allocations, interleaved,
        # all kept alive (independent placements), after the bench's own
        d0 = torch.from_numpy(frames.reshape(-1)).cuda()
        A = d0.repeat(rep)
        del d0
        size = A.numel()
        res.append(entry("A (bench allocation)", A))
        hip = C.CDLL("libamdhip64.so")
        for i in range(6):
            for name, flags in (("contiguous", 4), ("plain", 0)):
                p = C.c_void_p()
                rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(size), C.c_uint(flags))
                if rc:
                    res.append({"slab": "%s %d" % (name, i), "error": rc})
                    continue
                assert hip.hipMemcpy(p, C.c_void_p(A.data_ptr()), C.c_size_t(size), 3) == 0
                res.append(entry("%s %d" % (name, i), Raw(p.value)))
        with open(out_path, "w") as f:
            json.dump({"what": "many", "pkts": n, "results": res}, f, indent=1)
        return
    d0 = torch.from_numpy(frames.reshape(-1)).cuda()
    A = d0.repeat(rep)
    del d0
    size = A.numel()
    res.append(entry("A (bench allocation)", A))
    # hipExtMallocWithFlags: physically contiguous (best effort), and plain
    hip = C.CDLL("libamdhip64.so")
    raw = []
    for name, flags in (("D1 (hipDeviceMallocContiguous)", 4), ("E1 (hipExtMallocWithFlags 0)", 0),
                        ("D2 (hipDeviceMallocContiguous)", 4), ("E2 (hipExtMallocWithFlags 0)", 0),
                        ("D3 (hipDeviceMallocContiguous)", 4), ("E3 (hipExtMallocWithFlags 0)", 0)):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(size), C.c_uint(flags))
        if rc:
            res.append({"slab": name, "error": rc})
            continue
        raw.append(p)
        assert hip.hipMemcpy(p, C.c_void_p(A.data_ptr()), C.c_size_t(size), 3) == 0
        res.append(entry(name, Raw(p.value)))
    B = torch.empty_like(A)
    B.copy_(A)
    res.append(entry("B (second torch allocation)", B))
    res.append(entry("A again", A))
    # A's memory handed back and taken again
    del A
    torch.cuda.empty_cache()
    A2 = torch.empty_like(B)
    A2.copy_(B)
    res.append(entry("A2 (after A was freed)", A2))
    del A2
    for p in raw:
        hip.hipFree(p)
    torch.cuda.empty_cache()
    Cs = torch.empty(size + 4096, dtype=torch.uint8, device="cuda")
    for off in (0, 1024):
        v = Cs[off:off + size]
        v.copy_(B)
        res.append(entry("C + %d" % off, v))
    with open(out_path, "w") as f:
        json.dump({"what": __doc__.strip().splitlines()[0], "pkts": n, "results": res}, f,
                  indent=1)


if __name__ == "__main__":
    main()

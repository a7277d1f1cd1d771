#!/usr/bin/env python3
"""C4 WildcardMatch timed through a given build of libbessgpu.so (argv[1];
default the product library): 8 M IMIX packets, 100 K rules over 8 masks,
the header lines in a dense 64 B slab and the frames in 2 KB slots. Run once
per library in separate processes on one box to compare kernel versions.
Prints one JSON line."""
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
    n0, rep = 1 << 20, 8
    n = n0 * rep
    rk, rm, prio, gates, frames, flen = P.wm_workload(100000, n0, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    out = {"lib": os.path.basename(_lib.LIB_PATH)}
    try:  # the run-time compiled kernel, when the build has one
        t.jit_wait()
        out["jit"] = True
    except (_lib.BessGpuError, AttributeError):
        out["jit"] = False

    def timed(slab, stride, g):
        t.classify(slab, stride, n, 8192, g)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                t.classify(slab, stride, n, 8192, g)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 10)
        return round(best, 4), g.cpu().numpy().view(np.uint16)[:n0].copy()

    flags = int(os.environ.get("WM_AB_FLAGS", "0"), 0)
    h = torch.from_numpy(np.ascontiguousarray(frames[:, :64]).reshape(-1)).cuda().repeat(rep)
    g = torch.empty(n, dtype=torch.int16, device="cuda")
    ref = None
    for name, fl in (("default", 0), ("flags", flags)) if flags else (("default", 0),):
        with _lib.kernel_paths(fl):
            out[name + "_slab_ms"], gh = timed(h, 64, g)
        ref = gh if ref is None else ref
        out[name + "_same_as_default"] = bool((gh == ref).all())
    del h
    d = torch.from_numpy(frames.reshape(-1)).cuda().repeat(rep)
    for name, fl in (("default", 0), ("flags", flags)) if flags else (("default", 0),):
        with _lib.kernel_paths(fl):
            out[name + "_slots2k_ms"], g2 = timed(d, 2048, g)
        out[name + "_2k_same"] = bool((g2 == ref).all())
    out["gates_crc"] = int(np.bitwise_xor.reduce(ref.astype(np.uint64) * np.arange(1, n0 + 1, dtype=np.uint64)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""WildcardMatch at the batch sizes a bessd pipe slot holds (C4 rules: 100 K
over 8 masks, IMIX header lines in a dense 64 B slab): microseconds per
launch, back to back on one stream, for the tag-word kernel (default) and
the L2-probe kernel (BG_PATH_NO_LDS); gates compared. One JSON line per n."""
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
    n0 = 1 << 16
    rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n0, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    t.jit_wait()
    h = torch.from_numpy(np.ascontiguousarray(frames[:, :64]).reshape(-1)).cuda()
    g = torch.empty(n0, dtype=torch.int16, device="cuda")
    s = torch.cuda.Stream()
    for n in (256, 512, 1024, 2048, 4096, 16384, 65536):
        out = {"n": n}
        ref = None
        for name, fl in (("tags", 0), ("l2", 2)):
            with _lib.kernel_paths(fl), torch.cuda.stream(s):
                reps = max(20, min(400, (1 << 22) // n))
                for _ in range(5):
                    t.classify(h, 64, n, 8192, g, stream=s)
                s.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    t.classify(h, 64, n, 8192, g, stream=s)
                e1.record(s)
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / reps
            got = g.cpu().numpy().view(np.uint16)[:n].copy()
            ref = got if ref is None else ref
            out[name + "_us"] = round(us, 2)
            out[name + "_Mpps"] = round(n / us, 1)
            out[name + "_same"] = bool((got == ref).all())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

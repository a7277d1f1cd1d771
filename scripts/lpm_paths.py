#!/usr/bin/env python3
"""IPLookup kernel forms timed on the bench workload (16 M 64 B packets,
10 K routes, half the destinations inside a route; one process): the
default (DIR-16-8-8, tbl16 in LDS), DIR-16-8-8 with tbl16 in L2
(BG_PATH_NO_LDS) and DIR-24-8 (BG_PATH_LPM_DIR24). Gates must agree."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bess_amd import _lib as LB  # noqa: E402
from test_gpu_iplookup import build, dsts_inside, frames_to, routes  # noqa: E402


def main():
    n = 1 << 24
    rng = np.random.default_rng(0x5EED)
    rt = routes(10000, rng, 0.05)
    m, _ = build(rt, max_rules=20000, max_tbl8s=4096)
    dst = np.concatenate([dsts_inside(rt, n // 2, rng),
                          rng.integers(0, 1 << 32, n - n // 2, dtype=np.uint64)])
    rng.shuffle(dst)
    d = torch.from_numpy(frames_to(dst).reshape(-1)).cuda()
    g = torch.empty(n, dtype=torch.int16, device="cuda")
    res, ref = {}, None
    for name, fl in (("default_dir16_8_8_tbl16_lds", 0),
                     ("dir16_8_8_tbl16_l2", LB.BG_PATH_NO_LDS),
                     ("dir24_8", LB.BG_PATH_LPM_DIR24)):
        with LB.kernel_paths(fl):
            m.process_device(d, 64, n, g)
            torch.cuda.synchronize()
            got = g.cpu().numpy()
            ref = got if ref is None else ref
            assert (got == ref).all(), name
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    m.process_device(d, 64, n, g)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            res[name] = round(min(ts), 4)
    print(json.dumps({"lpm_paths_ms": res}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""ACL kernel forms timed on the bench workload (16 M 64 B packets, 100 and
1000 rules, and 1000 / 3000 / 8000 rules with the catch-all rules removed;
one process): the default (the decision trees), the rule scan from LDS
(BG_PATH_ACL_LDS), the scan with scalar rule loads (BG_PATH_ACL_SCAN), the
per-dimension bit vectors (BG_PATH_ACL_BV). Gates must agree across forms."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bess_amd import _lib as LB  # noqa: E402

if len(sys.argv) > 1:  # another build of the library (A/B on one box)
    LB.LIB_PATH = os.path.abspath(sys.argv[1])
from bess_amd.modules import ACL  # noqa: E402
from test_gpu_acl import workload  # noqa: E402


def main():
    n = 1 << 24
    out = {}
    g = torch.empty(n, dtype=torch.int16, device="cuda")
    for nr, full in ((100, 1), (1000, 1), (1000, 0), (3000, 0), (8000, 0)):
        rules, frames = workload(nr, n, seed=nr)
        if not full:  # no rule that ends every wave's scan early
            rules = [r for r in rules if r.get("src_ip") or r.get("dst_ip")]
        d = torch.from_numpy(frames.reshape(-1)).cuda()
        m = ACL(rules=rules)
        res = {}
        ref = None
        forms = [("default", 0), ("lds_scan", LB.BG_PATH_ACL_LDS),
                 ("scalar_scan", LB.BG_PATH_ACL_SCAN), ("bitvec", LB.BG_PATH_ACL_BV)]
        if nr > 1000:
            forms = forms[:2]  # the scans take ~ms per launch there
        for name, fl in forms:
            with LB.kernel_paths(fl):
                m.process_device(d, 64, n, g)
                torch.cuda.synchronize()
                got = g.cpu().numpy()
                if ref is None:
                    ref = got
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
        out["rules_%d%s" % (nr, "" if full else "_no_catch_all")] = res
        del d
    print(json.dumps({"acl_paths_ms": out}))


if __name__ == "__main__":
    main()

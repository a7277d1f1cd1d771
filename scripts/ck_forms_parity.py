"""Every checksum kernel form of the measurement build (libbessgpu_ab.so,
BG_CK_TILED) against the oracle on the parity suite's frames: the edge
frames of tests/test_gpu_parity.py (VLAN/QinQ, IHL < 5 and > 5, bad UDP/TCP
lengths, all-ones payloads, UDP checksum 0) in modes 1/2/3, calc and verify,
and C3-style workloads of 60/590/1496 B frames. Prints one JSON line: form
-> number of failing cases (0 = bit-exact everywhere)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bess_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", "bin", "libbessgpu_ab.so")
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_parity import edge_frames  # noqa: E402

FORMS = {"default": 0, "reload_d2": 9, "words_d2": 8, "stash_d2": 7, "words_nt": 14}


def run(frames, mode, verify, dev):
    n = frames.shape[0]
    ref = frames.copy()
    ipw, l4w = O.cksum_process(ref, 2048, n, mode, verify)
    d = torch.from_numpy(frames.reshape(-1).copy()).to(dev)
    ipg = torch.zeros(n, dtype=torch.int16, device=dev)
    l4g = torch.zeros(n, dtype=torch.int16, device=dev)
    F.cksum(d, 2048, n, mode, verify, ipg, l4g)
    torch.cuda.synchronize()
    out = d.cpu().numpy().reshape(n, 2048)
    ok = (out == ref).all()
    if mode & 1:
        ok = ok and (ipg.cpu().numpy().view(np.uint16) == ipw).all()
    if mode & 2:
        ok = ok and (l4g.cpu().numpy().view(np.uint16) == l4w).all()
    return bool(ok)


def main():
    assert _lib.lib().bg_is_ab_build() == 1
    dev = torch.device("cuda:0")
    cases = []
    for verify in (False, True):
        fr = edge_frames()
        if verify:
            O.cksum_process(fr[::2], 2048, fr[::2].shape[0], 3, False)
        for mode in (1, 2, 3):
            cases.append(("edges_m%d_v%d" % (mode, verify), fr, mode, verify))
    for L in (60, 590, 1496):
        fr = P.cksum_workload(8192, frame_len=L, seed=L)
        for mode, verify in ((3, False), (2, True), (1, True)):
            cases.append(("wl%d_m%d_v%d" % (L, mode, verify), fr, mode, verify))
    res = {}
    for form, v in FORMS.items():
        os.environ["BG_CK_TILED"] = str(v)
        bad = [name for name, fr, mode, verify in cases if not run(fr, mode, verify, dev)]
        res[form] = {"cases": len(cases), "failed": bad}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

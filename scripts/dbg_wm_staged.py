"""Diagnose the WildcardMatch launch-mode pipe mismatch with two 4-byte attr
fields (tests/test_gpu_pipe.py::test_pipe_rebind_permuted_attr_offsets):
which datapath (ring, launch + AOT tags, launch + no tags, sync host path)
disagrees with the oracle, and how."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from bess_amd import _lib as LB  # noqa: E402
from bess_amd.modules import Pipe, WildcardMatch  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_attr_fields import META_OFF, STRIDE, slots  # noqa: E402

fields = [{"attr_name": "foo", "num_bytes": 4}, {"attr_name": "bar", "num_bytes": 4},
          {"offset": 26, "num_bytes": 2}]
lay = {"foo": 8, "bar": 12}
n = 20000
f = slots(n, 71)
frames = np.ascontiguousarray(f[:, :META_OFF])
meta = np.ascontiguousarray(f[:, META_OFF:])
heads = frames.ctypes.data + META_OFF * np.arange(n, dtype=np.uintp)
metas = meta.ctypes.data + (STRIDE - META_OFF) * np.arange(n, dtype=np.uintp)


def build(nr):
    rng = np.random.default_rng(72)
    o, m = O.OracleWildcardMatch(fields=fields), WildcardMatch(fields=fields)
    mk = [{"value_bin": b"\xff" * 4}, {"value_bin": b"\xff" * 4}, {"value_bin": b"\xff\xff"}]
    for i in rng.choice(n, nr, replace=False):
        vals = [{"value_bin": f[i, META_OFF + 8:META_OFF + 12].tobytes()},
                {"value_bin": f[i, META_OFF + 12:META_OFF + 16].tobytes()},
                {"value_bin": f[i, 26:28].tobytes()}]
        g = int(rng.integers(0, 64))
        o.add(values=vals, masks=mk, gate=g, priority=1)
        m.add(values=vals, masks=mk, gate=g, priority=1)
    m.bind_meta(-1, lay)
    return o, m


def run_pipe(m):
    pipe = Pipe(m, batch=1024, depth=3)
    cs, gs = [], []
    for i in range(0, n, 32):
        idx = np.arange(i, min(n, i + 32), dtype=np.uintp)
        pipe.submit(heads[idx], cookies=idx, metas=metas[idx])
        c, g = pipe.poll()
        cs.append(c)
        gs.append(g)
    c, g = pipe.drain()
    pipe.close()
    got = np.empty(n, np.uint16)
    got[np.concatenate(cs + [c]).astype(np.int64)] = np.concatenate(gs + [g])
    return got


for nr in (500, 1500, 5000):
    o, m = build(nr)
    want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=lay)
    info = None
    for name, flags in (("ring", 0), ("launch", LB.BG_PATH_PIPE_NO_RING),
                        ("launch_nojit", LB.BG_PATH_PIPE_NO_RING | LB.BG_PATH_WM_NO_JIT),
                        ("launch_notags", LB.BG_PATH_PIPE_NO_RING | LB.BG_PATH_WM_NO_TAGS)):
        with LB.kernel_paths(flags):
            got = run_pipe(m)
            try:
                info = m.table_info() if hasattr(m, "table_info") else None
            except Exception:
                info = None
        bad = np.nonzero(got != want)[0]
        print(nr, name, "mismatch", len(bad), "hits", int((want != O.DROP_GATE).sum()),
              "sample", [(int(i), int(got[i]), int(want[i])) for i in bad[:6]], info, flush=True)
    with LB.kernel_paths(0):
        g2 = m.process_meta(heads, metas)
    bad = np.nonzero(g2 != want)[0]
    print(nr, "sync", "mismatch", len(bad), [(int(i), int(g2[i]), int(want[i])) for i in bad[:6]],
          flush=True)

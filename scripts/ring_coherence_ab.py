"""A/B of the persistent ring's per-ticket coherence (bg_ring_set_coherence;
the measurement build's BG_RING_COHERENCE = 1 + bit0 system-scope acquire +
bit1 release on the done word): 32..1024-packet tickets from 1 and 16
submitters over device-resident frames, and the ExactMatch pipe on the ring
(host snbufs, 16 workers). One JSON line per mode.

    python scripts/ring_coherence_ab.py > gpurun_out/ring_coh.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "scripts", "bin", "libbessgpu_ab.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bess_amd import flowtable as F, packets as P  # noqa: E402
from bess_amd.modules import ExactMatch, Pipe  # noqa: E402

assert _lib.lib().bg_is_ab_build() == 1
npk = 4 << 20
keys, gates, frames = P.em_workload(1000, npk, seed=0x5EED)
d = torch.from_numpy(frames.reshape(-1)).cuda()
dg = torch.empty(npk, dtype=torch.int16, device="cuda")
t = F.EmTable(P.em_fields_5tuple())
t.add_many(keys, gates)
t.sync(0)
m = ExactMatch(fields=[{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE])
cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
for k, g in zip(keys, gates):
    kb = k.tobytes()
    m.add(fields=[{"value_bin": kb[a:c]} for a, c in cut], gate=int(g))
nh = 1 << 18
snb = np.zeros((nh, 2624), np.uint8)
snb[:, 512:576] = frames[:nh]
heads = snb.ctypes.data + 512 + 2624 * np.arange(nh, dtype=np.uintp)
for mode in (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")):
    os.environ["BG_RING_COHERENCE"] = str(mode)
    out = {"mode": mode, "sys_acquire": bool((mode - 1) & 1), "release": bool((mode - 1) & 2)}
    for T in (1, 16):
        ring = F.Ring(t, slots=4096, lanes=T)
        ring.set_coherence(1, 1)  # (overridden by the knob)
        for B in (32, 256, 1024):
            ring.run_lanes(d, 64, npk, B, 8192, dg, T)
            best = min(ring.run_lanes(d, 64, npk, B, 8192, dg, T) for _ in range(3))
            out["T%d_B%d_Mpps" % (T, B)] = round(npk / best / 1e6, 1)
        ring.close()
    # the pipe on the module's ring: 16 worker threads over host snbufs (a
    # rule re-added: a new ring, created under this mode's knob)
    kb = keys[0].tobytes()
    m.add(fields=[{"value_bin": kb[a:c]} for a, c in cut], gate=int(gates[0]))
    import threading
    pipes = [Pipe(m, batch=1024, depth=8) for _ in range(16)]
    for p in pipes:
        p.run(heads[:4096])
    outs = [None] * 16
    t0 = time.perf_counter()
    ths = [threading.Thread(target=lambda i=i: outs.__setitem__(i, pipes[i].run(
        heads[nh * i // 16: nh * (i + 1) // 16]))) for i in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    out["pipe16_Mpps"] = round(nh / (time.perf_counter() - t0) / 1e6, 1)
    for p in pipes:
        p.close()
    print(json.dumps(out), flush=True)

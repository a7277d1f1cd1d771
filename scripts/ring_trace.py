#!/usr/bin/env python3
"""Where a persistent-ring ticket's time goes (A/B build, BG_RING_TRACE):
1 M resident 64 B packets in 32-packet tickets from T submitter threads on
T lanes; the kernel stamps each ticket (s_memrealtime, 100 MHz) when a
workgroup claims it, sees it published, has read its descriptor, has its
gates stored, and has written its done word. Prints one JSON line per T
with the medians of each interval and the ticket rate.
Usage: python scripts/ring_trace.py [--wm] [--batch=B] [T ...]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", "bin", "libbessgpu_ab.so")
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def main():
    args = sys.argv[1:]
    wm = "--wm" in args  # C4's WildcardMatch table (bg_wm_ring_create)
    args = [a for a in args if a != "--wm"]
    B = 32
    for a in list(args):
        if a.startswith("--batch="):
            B = int(a.split("=")[1])
            args.remove(a)
    ts = [int(x) for x in args] or [1, 4, 16]
    n = 1 << 20
    if wm:
        rk, rm, prio, wg, wf, _ = P.wm_workload(100000, n, stride=2048)
        t = F.WmTable(P.FIVE_TUPLE)
        for k, m, p, g in zip(rk, rm, prio, wg):
            t.add(k.tobytes(), m.tobytes(), int(p), int(g))
        frames = np.ascontiguousarray(wf[:, :64])
    else:
        keys, gates, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=77)
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
    d_frames = torch.from_numpy(frames.reshape(-1)).cuda()
    d_g = torch.zeros(n, dtype=torch.int16, device="cuda")
    L = _lib.lib()
    L.bg_ring_trace.restype = C.c_int
    L.bg_ring_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    for T in ts:
        per_lane = n // T // B
        os.environ["BG_RING_TRACE"] = str(per_lane)
        ring = F.Ring(t, slots=4096, lanes=T)
        ring.set_coherence(1, 0)  # as the pipes and the bench sweep use it
        os.environ.pop("BG_RING_TRACE")
        ring.run_lanes(d_frames, 64, n, B, 8192, d_g, T)  # warm (stamps overwritten)
        dt = ring.run_lanes(d_frames, 64, n, B, 8192, d_g, T)
        dev = ring.desc_in_device()
        buf = np.zeros(T * per_lane * 5, np.uint64)
        tn = L.bg_ring_trace(ring.h, buf.ctypes.data, buf.size)
        ring.close()
        st = buf.reshape(T, tn, 5).astype(np.float64) * 10.0  # ns
        ok = (st > 0).all(axis=2)
        s = st[ok]
        iv = {"claim_to_seen_us": s[:, 1] - s[:, 0], "seen_to_desc_us": s[:, 2] - s[:, 1],
              "desc_to_stored_us": s[:, 3] - s[:, 2], "stored_to_done_us": s[:, 4] - s[:, 3]}
        out = {"table": "wm" if wm else "em", "submitters": T, "desc_in_device": dev, "tickets": int(ok.sum()), "batch": B,
               "Mpps": round(n / dt / 1e6, 1)}
        for k, v in iv.items():
            out[k] = {"p50": round(float(np.median(v)) / 1e3, 2),
                      "p90": round(float(np.percentile(v, 90)) / 1e3, 2)}
        # GPU-side rate: tickets done per us over the middle of the run
        done = np.sort(s[:, 4])
        m0, m1 = done[len(done) // 10], done[len(done) * 9 // 10]
        out["gpu_tickets_per_us_mid80"] = round(0.8 * len(done) / ((m1 - m0) / 1e3), 2)
        # in flight: tickets between seen and done at the midpoint
        mid = (m0 + m1) / 2
        out["tickets_in_service_at_mid"] = int(((s[:, 1] <= mid) & (s[:, 4] >= mid)).sum())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

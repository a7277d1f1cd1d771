"""Persistent-ring latency and rate by where a ticket's frames and gates
live (device memory, or pinned host memory the kernel reads over PCIe, as a
ring-mode pipe's staged windows are): one ticket submitted and waited for
(median of 200), and back-to-back tickets on one lane. Prints JSON lines.
Usage: python scripts/ring_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def main():
    n = 1 << 20
    keys, gates, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=77)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    # staged windows as a pipe stages them: frame bytes [23, 39) in 16 B
    win = np.ascontiguousarray(frames[:, 23:39])
    ref = None
    for where in ("device", "host"):
        for what, data, stride, off in (("frames64", frames, 64, 0),
                                        ("windows16", win, 16, 23)):
            src = torch.from_numpy(data.reshape(-1).copy())
            src = src.cuda() if where == "device" else src.pin_memory()
            g = torch.zeros(n, dtype=torch.int16)
            g = g.cuda() if where == "device" else g.pin_memory()
            r = F.Ring(t, slots=4096, lanes=1, win_off=off)
            res = {"frames_and_gates_in": where, "slot": what}
            for b in (32, 1024, 4096):
                lat = []
                for i in range(200):
                    t0 = time.perf_counter()
                    k = r.submit(src, stride, b, 8192, g, offset=(i * b) % (n - b))
                    r.wait(k)
                    lat.append((time.perf_counter() - t0) * 1e6)
                res["latency_us_%d" % b] = round(float(np.median(lat)), 1)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.run(src, stride, n, b, 8192, g)
                res["Mpps_back_to_back_%d" % b] = round(n / (time.perf_counter() - t0) / 1e6, 1)
            got = g.cpu().numpy().view(np.uint16).copy()
            if ref is None:
                ref = got
            res["same_gates_as_first"] = bool((got == ref).all())
            r.close()
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

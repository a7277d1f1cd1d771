#!/usr/bin/env python3
"""The ring sweep's 16-submitter rows at large tickets:
every repetition, not the best of three, with the cgroup's CPU throttling
(cpu.stat nr_throttled / throttled_usec) read around each one and the
process's voluntary / involuntary context switches (getrusage, all
threads). C2's slab (1000 rules, 16 M resident 64 B packets) as in
bench.py's em_sweep.
Usage: python scripts/ring_dip_probe.py OUT.json [reps]"""
import json
import os
import resource
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            d = dict(line.split() for line in f if line.strip())
        return {k: int(v) for k, v in d.items()}
    except OSError:
        return {}


def main():
    out = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    n = 16 << 20
    keys, gates, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=0x5EED)
    d_frames = torch.from_numpy(frames.reshape(-1)).to(dev)
    del frames
    d_gates = torch.empty(n, dtype=torch.int16, device=dev)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    t.sync(0)
    torch.cuda.synchronize()
    res = {"what": "ring sweep rows, every repetition (4 passes per thread each)",
           "cpu_max": open("/sys/fs/cgroup/cpu.max").read().strip()
           if os.path.exists("/sys/fs/cgroup/cpu.max") else None,
           "runs": []}
    for T in (4, 16):
        ring = F.Ring(t, slots=4096, lanes=T)
        ring.set_coherence(1, 0)
        for B in (256, 1024, 2048, 4096):
            ring.run_lanes(d_frames, 64, n, B, 8192, d_gates, T)  # warm
            for i in range(reps):
                c0, r0 = cpu_stat(), resource.getrusage(resource.RUSAGE_SELF)
                w0 = time.perf_counter()
                dt = ring.run_lanes(d_frames, 64, n, B, 8192, d_gates, T, reps=4)
                w1 = time.perf_counter()
                c1, r1 = cpu_stat(), resource.getrusage(resource.RUSAGE_SELF)
                res["runs"].append({
                    "T": T, "B": B, "i": i, "Mpps": round(n / dt / 1e6, 1),
                    "wall_ms": round((w1 - w0) * 1e3, 3),
                    "throttled": c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0),
                    "throttled_us": c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0),
                    "cpu_ms": round((c1.get("usage_usec", 0) - c0.get("usage_usec", 0)) / 1e3, 2),
                    "nvcsw": r1.ru_nvcsw - r0.ru_nvcsw, "nivcsw": r1.ru_nivcsw - r0.ru_nivcsw})
                print(json.dumps(res["runs"][-1]), flush=True)
        launches, blocks = ring.info()
        res["launches_T%d" % T] = launches
        ring.close()
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

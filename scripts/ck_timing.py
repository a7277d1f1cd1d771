"""C3's checksum launch timed several ways in one process (product library):
the bench leg's loop (W warm-ups, K steps between two events), variants.py's
(rounds of 40 launches), and per-launch events -- to tell a timing-method
difference from a kernel difference. Prints one JSON line."""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if len(sys.argv) > 1 and sys.argv[1].startswith("ab="):
    # PMC passes of an A/B form: `ck_timing.py ab=8` launches
    # cksum_kernel<3, 2> from the measurement build, three times
    os.environ["BG_CK_TILED"] = sys.argv[1][3:]
    from bess_amd import _lib  # noqa: E402
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "bin", "libbessgpu_ab.so")
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402


def loop(fn, warm, reps):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda:0")
    n = 1 << 20
    frames = P.cksum_workload(n, frame_len=1496, stride=2048)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    del frames
    g = torch.empty(n, dtype=torch.int16, device=dev)
    fn = lambda: F.cksum(d, 2048, n, 3, False, None, g)  # noqa: E731
    if len(sys.argv) > 1:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(json.dumps({"launches": 3, "variant": sys.argv[1]}))
        return
    out = {}
    out["bench_5_20"] = round(loop(fn, 5, 20), 4)
    out["bench_100_200"] = round(loop(fn, 100, 200), 4)
    out["variants_5x40"] = [round(loop(fn, 1, 40), 4) for _ in range(5)]
    ev = []
    for _ in range(20):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ev.append(a.elapsed_time(b))
    out["single_launch_median"] = round(statistics.median(ev), 4)
    # the same slab re-allocated (a different placement)
    d2 = d.clone()
    del d
    torch.cuda.synchronize()
    fn2 = lambda: F.cksum(d2, 2048, n, 3, False, None, g)  # noqa: E731
    out["clone_5_20"] = round(loop(fn2, 5, 20), 4)
    # host-side cost of one call (no sync)
    import time
    t0 = time.perf_counter()
    for _ in range(200):
        fn2()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    out["host_us_per_call"] = round((t1 - t0) / 200 * 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

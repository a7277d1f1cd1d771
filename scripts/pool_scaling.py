#!/usr/bin/env python3
"""The bounded-pool WildcardMatch pipeline (bench.py run_plugin_pool) by
worker count: the GPU plugin and the restated reference in the same
harness, one drive process per count. One JSON line per count."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import packets as P, pb  # noqa: E402


def main():
    drive = os.environ.get("DRIVE") or os.path.join(ROOT, "tests", "bessd_shell", "build", "drive")
    counts = [int(x) for x in sys.argv[1:]] or [4, 8, 12, 16]
    n, nr = 1 << 17, 100000
    fields = [{"offset": o, "num_bytes": sz} for o, sz in P.FIVE_TUPLE]
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    rk, rm, prio, wg, frames, _ = P.wm_workload(nr, n, stride=2048)
    base = ["create WildcardMatch " + pb.dict_to_protobuf(
        pb.WildcardMatchArg, {"fields": fields}).SerializeToString().hex()]
    for k, mk, p, g in zip(rk, rm, prio, wg):
        kb, mb = k.tobytes(), mk.tobytes()
        a = dict(gate=int(g), priority=int(p), values=[{"value_bin": kb[x:y]} for x, y in cut],
                 masks=[{"value_bin": mb[x:y]} for x, y in cut])
        base.append("cmd add " + pb.dict_to_protobuf(pb.WildcardMatchCommandAddArg, a)
                    .SerializeToString().hex())
    base += ["connect %d" % g for g in range(64)]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "f.bin")
        frames.tofile(path)
        wp = [os.path.join(td, x) for x in "kmpg"]
        for arr, pth, dt in zip((rk, rm, prio, wg), wp, (np.uint8, np.uint8, np.int32, np.uint16)):
            np.ascontiguousarray(arr, dtype=dt).tofile(pth)
        base += ["cpu_wm %s %s %s %s %d" % (*wp, nr), "frames %s 2048 %d" % (path, n),
                 "pool 262144"]
        for nw in counts:
            sc = base + ["pipeline %d 1 0 0 0" % nw, "sleep 3000", "pipeline %d 40 0 0 0" % nw,
                         "pipeline_cpu %d 1" % nw, "pipeline_cpu %d 40" % nw]
            r = subprocess.run([drive, "run"],
                               input="\n".join(sc) + "\n", capture_output=True, text=True,
                               timeout=600)
            st = [x.split() for x in r.stdout.splitlines() if x.startswith("pipeline")]
            cyc = [x for x in r.stdout.splitlines() if x.startswith("cycles")]
            out = {"drive": os.path.basename(drive), "workers": nw, "rc": r.returncode}
            if len(st) >= 4:
                out.update(gpu_Mpps=float(st[1][1]), cpu_Mpps=float(st[3][1]),
                           gpu_cycles=cyc[1][7:] if len(cyc) > 1 else "",
                           cpu_cycles=cyc[3][7:] if len(cyc) > 3 else "")
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

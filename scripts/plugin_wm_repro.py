"""Repro of the WildcardMatch plugin leg on a bounded pool (bench.py
run_plugin_pool), with the driver's crash backtrace on stderr."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bess_amd import packets as P, pb  # noqa: E402

n, nr = 1 << 17, int(sys.argv[1]) if len(sys.argv) > 1 else 100000
fields = [{"offset": o, "num_bytes": sz} for o, sz in P.FIVE_TUPLE]
cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
rk, rm, prio, wg, frames, _ = P.wm_workload(nr, n, stride=2048)
script = ["create WildcardMatch " + pb.dict_to_protobuf(
    pb.WildcardMatchArg, {"fields": fields}).SerializeToString().hex()]
for k, mk, p, g in zip(rk, rm, prio, wg):
    kb, mb = k.tobytes(), mk.tobytes()
    a = dict(gate=int(g), priority=int(p), values=[{"value_bin": kb[x:y]} for x, y in cut],
             masks=[{"value_bin": mb[x:y]} for x, y in cut])
    script.append("cmd add " + pb.dict_to_protobuf(pb.WildcardMatchCommandAddArg, a)
                  .SerializeToString().hex())
script += ["connect %d" % g for g in range(64)]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
path = os.path.join(ROOT, "gpurun_out", "wmf.bin")
frames.tofile(path)
script += ["frames %s 2048 %d" % (path, n)] + sys.argv[2:]
r = subprocess.run([os.path.join(ROOT, "tests", "bessd_shell", "build", "drive"), "run"],
                   input="\n".join(script) + "\n", capture_output=True, text=True, timeout=300)
os.remove(path)
print("rc", r.returncode)
print("\n".join(x[:200] for x in r.stdout.splitlines() if not x.startswith("rc 0")))
print(r.stderr[-4000:])

#!/usr/bin/env python3
"""DESIGN.md §6's measurement table from one bench line (the JSON bench.py
prints), so the record quotes a measured line and nothing else.

usage: python scripts/design_table.py profiles/r03_bench_line.json"""
import json
import sys


def frac(r):
    return "%.2f" % r["frac"] if r and r.get("frac") is not None else "--"


def tr(r, bpp):
    """PMC traffic per launch over the algorithmic bytes"""
    if not r or not r.get("traffic_bytes_per_launch"):
        return "--"
    return "%.2f" % (r["traffic"] / r["achieved"]) if r.get("traffic") else "--"


def cpu(c):
    if not c:
        return "--"
    v = c["value"]
    s = ("%.2f Gpps" % (v / 1e3)) if v >= 1000 else ("%.0f Mpps" % v)
    return "%s (%d thr; %.1f Mpps/thr)" % (s, c["cores"], c.get("single_core_mpps", v))


def rate(mpps):
    return ("%.1f Gpps" % (mpps / 1e3)) if mpps >= 1000 else ("%.0f Mpps" % mpps)


def main():
    line = open(sys.argv[1]).read().strip().splitlines()[-1]
    d = json.loads(line)
    # (round 5 on: the §8f modules under "modules_8f", C1 at the top level)
    x = dict(d.get("modules_8f", {}))
    x.update(d["extra_configs"])
    if "C1" in d:
        x["C1"] = d["C1"]
    rows = []
    rows.append(("**C2** EM, 1 K rules (headline)", "%.4f ms" % d["roofline"]["kernel_ms"],
                 rate(d["value"]), "**%s**" % frac(d["roofline"]), tr(d["roofline"], 66),
                 cpu(d["cpu_baseline"])))
    c1 = x.get("C1")
    if c1:
        rows.append(("C1 Source -> EM (1 rule) -> Sink (CPU path)", "--", "--", "--", "--",
                     cpu(c1["cpu_baseline"])))
    c3 = x.get("C3")
    if c3:
        rows.append(("C3 IP+L4 checksum, 1 M x 1496 B", "%.4f ms" % c3["ms_per_step"],
                     rate(c3["Mpps"]), frac(c3["roofline"]), tr(c3["roofline"], 1502),
                     cpu(c3.get("cpu_baseline"))))
    c4 = x.get("C4")
    if c4:
        s2 = c4["slots_2k"]
        rows.append(("C4 WM, 100 K rules, 8 masks, 8 M IMIX: header slab / 2 KB slots "
                     "(run-time compiled kernel)",
                     "%.4f / %.4f ms" % (c4["ms_per_step"], s2["ms_per_step"]),
                     "%s / %s" % (rate(c4["Mpps"]), rate(s2["Mpps"])),
                     "%s / %s" % (frac(c4["roofline"]), frac(s2["roofline"])),
                     "%s / %s" % (tr(c4["roofline"], 66), tr(s2["roofline"], 66)),
                     cpu(c4.get("cpu_baseline"))))
        a = c4.get("ahead_of_time")
        if a:
            rows.append(("C4, the ahead-of-time kernel (same process)",
                         "%.4f / %.4f ms" % (a["ms_per_step"], a["slots_2k_ms_per_step"]),
                         "--", "--", "--", "--"))
    em15 = x.get("EM_1500B")
    if isinstance(em15, dict):
        mc = em15.get("measured_ceiling") or {}
        rows.append(("EM, 1 K rules, 1500 B packets (1496 B frames in 2 KB slots, 4 M)",
                     "%.4f ms" % em15["ms_per_step"], rate(em15["Mpps"]),
                     "%s (%.2f of s2k32)" % (frac(em15["roofline"]), mc.get("frac_of_ceiling", 0)),
                     tr(em15["roofline"], 66), cpu(em15.get("cpu_baseline"))))
    c5 = x.get("C5")
    if c5:
        rows.append(("C5 EM, 1 M rules (1 GPU), table in L2/MALL", "%.4f ms" % c5["ms_per_step"],
                     rate(c5["Mpps"]), frac(c5["roofline"]), tr(c5["roofline"], 66),
                     cpu(c5.get("cpu_baseline"))))
    h = x.get("HashLB")
    if h:
        rows.append(("HashLB l4, 8 gates", "%.4f ms" % h["l4"]["ms_per_step"],
                     rate(h["l4"]["Mpps"]), frac(h["l4"]["roofline"]),
                     tr(h["l4"]["roofline"], 66), cpu(h["l4"].get("cpu_baseline"))))
        f = h.get("fields_5tuple")
        if f:
            rows.append(("HashLB fields (5-tuple)", "%.4f ms" % f["ms_per_step"],
                         rate(f["Mpps"]), frac(f["roofline"]), tr(f["roofline"], 66),
                         cpu(f.get("cpu_baseline"))))
    acl = x.get("ACL")
    if acl:
        for k, lab in (("rules_100", "100"), ("rules_1000", "1000")):
            if k in acl:
                r = acl[k]
                rows.append(("ACL, %s rules (decision trees)" % lab, "%.4f ms" % r["ms_per_step"],
                             rate(r["Mpps"]), frac(r["roofline"]), tr(r["roofline"], 66),
                             cpu(r.get("cpu_baseline"))))
    for name, lab, bpp in (("IPLookup", "IPLookup, 10 K routes (DIR-16-8-8, tbl16 in LDS)", 66),
                           ("UpdateTTL", "UpdateTTL (in place)", 130),
                           ("StaticNAT", "StaticNAT, 16 pairs, 50 % translated (in place)", 130),
                           ("NAT", "NAT, established flows, 64 K mappings (in place)", 130),
                           ("Rewrite", "Rewrite, 4 templates of 60 B, 192 B slots (writes)", 70)):
        r = x.get(name)
        if r and "ms_per_step" in r:
            rows.append((lab, "%.4f ms" % r["ms_per_step"], rate(r["Mpps"]),
                         frac(r.get("roofline")), tr(r.get("roofline"), bpp),
                         cpu(r.get("cpu_baseline"))))
    print("| Workload (16 M x 64 B resident unless noted) | Kernel / step | Rate | HBM roofline "
          "frac | PMC traffic / algorithmic | CPU baseline (oracle on the box's leased threads) |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print("| " + " | ".join(r) + " |")
    sw = d.get("batch_sweep_mpps")
    if sw:
        print()
        print("C2 batch sweep (Mpps by packets per batch; resident packets):")
        print()
        sizes = sorted(sw["stream"], key=int)
        print("| path | " + " | ".join(sizes) + " |")
        print("|---|" + "---|" * len(sizes))
        for k in ("stream", "graph", "persistent", "persistent_4sub", "persistent_16sub"):
            if k in sw:
                print("| %s | " % k + " | ".join("%.0f" % sw[k][s] for s in sizes) + " |")


if __name__ == "__main__":
    main()

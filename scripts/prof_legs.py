#!/usr/bin/env python3
"""A kernel trace per bench leg, and the timed launches' own row per leg.

    python scripts/prof_legs.py run OUTDIR [leg ...]     (on the GPU box)
    python scripts/prof_legs.py summary OUTDIR > profiles/rNN_kernels.md

`run` traces each leg in a process of its own (rocprofv3 --kernel-trace
--stats around `bench.py` with the driver's --steps 20 --warmup 5), so
legs that launch the same kernel instantiation (C2 and C5 are both
em_slab_kernel<2, 2> on 512 workgroups) never share a row. `summary` takes
the leg's kernel from its trace and splits its dispatches: the last K are
the leg's timed launches (K = --steps for the headline, bench.py
leg_steps() = max(steps, 100) for the other section-8 configurations, 10
for the section-8f modules: nothing of the leg's kernel is launched after
its timed region), the rest are its parity check,
clock_settle and warm-up. The timed rows' average is what the bench line's
HIP-event time must agree with; the table prints both and their ratio.
"""
import csv
import glob
import json
import os
import subprocess
import sys

STEPS, WARMUP = 20, 5
# leg: (bench arguments, kernel name substring, where the leg's ms sits in
# its JSON line, timed launches)
LEGS = {
    "c2": ("--no-extra --no-cpu", "em_slab_kernel", ("roofline", "kernel_ms"), STEPS),
    "c3": ("--only cksum --no-cpu", "cksum_kernel", ("ms_per_step",), 100),
    "em1500": ("--only em1500 --no-cpu", "em_pair_kernel", ("ms_per_step",), 100),
    "c4_slab": ("--only wm --wm-layout slab --no-cpu", "bg_wm_jit", ("ms_per_step",), 100),
    "c4_2k": ("--only wm --wm-layout 2k --no-cpu", "bg_wm_jit",
              ("slots_2k", "ms_per_step"), 100),
    "c5": ("--only c5 --no-cpu", "em_slab_kernel", ("ms_per_step",), 100),
    # the section-8f modules: 10 timed launches each (bench.py _time_steps)
    "hashlb": ("--only hashlb --no-cpu", "line_slab_kernel<HlbFieldsOp",
               ("fields_5tuple", "ms_per_step"), 10),
    "acl": ("--only acl --no-cpu", "AclTreeOp", ("rules_1000", "ms_per_step"), 10),
    "iplookup": ("--only iplookup --no-cpu", "Lpm16LdsOp", ("ms_per_step",), 10),
    "ttl": ("--only ttl --no-cpu", "TtlOp", ("ms_per_step",), 10),
    "nat": ("--only nat --no-cpu", "NatOp", ("ms_per_step",), 10),
    "dnat": ("--only dnat --no-cpu --no-churn", "dnat_fused_slab_kernel", ("ms_per_step",), 10),
    "rewrite": ("--only rewrite --no-cpu", "rewrite_kernel", ("ms_per_step",), 100),
}


def run(out, legs):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(out, exist_ok=True)
    for leg in legs:
        args = LEGS[leg][0].split() + ["--steps", str(STEPS), "--warmup", str(WARMUP)]
        cmd = ["timeout", "-k", "10", "300", "rocprofv3", "--kernel-trace", "--stats",
               "--output-format", "csv", "-d", os.path.join(out, "prof_" + leg), "-o", leg,
               "--", sys.executable, os.path.join(root, "bench.py")] + args
        with open(os.path.join(out, leg + ".out"), "w") as fo, \
                open(os.path.join(out, leg + ".err"), "w") as fe:
            rc = subprocess.call(cmd, stdout=fo, stderr=fe)
        print("%s rc=%d" % (leg, rc), flush=True)
        if rc != 0:  # a fault, an abort or a time limit: nothing more on the GPU
            return rc
    return 0


def leg_line(out, leg):
    """the leg's JSON line: stdout for the headline, the last JSON line of
    stderr for an --only leg"""
    for name in (leg + ".out", leg + ".err"):
        try:
            lines = open(os.path.join(out, name)).read().splitlines()
        except OSError:
            continue
        for ln in reversed(lines):
            ln = ln.strip()
            if ln.startswith("{"):
                try:
                    return json.loads(ln)
                except ValueError:
                    pass
    return None


def dig(d, path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def short_name(name):
    name = name.replace("bg::(anonymous namespace)::", "").replace("bg::", "")
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, c in enumerate(name):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0:
            return name[:i].replace("> >", ">>")
    return name


def summary(out):
    print("Per bench leg (one rocprofv3 process each, `python bench.py <args> --steps %d "
          "--warmup %d`): the leg's kernel, its full-size dispatches, and the last K of "
          "them -- the leg's timed launches -- against the leg's HIP-event ms in its own "
          "JSON line.\n" % (STEPS, WARMUP))
    print("| leg | kernel | blocks | dispatches | K timed | timed avg us | timed median us "
          "| timed min us | other dispatches avg us | line ms | timed avg / line |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for leg, (_, pat, path, k) in LEGS.items():
        traces = glob.glob(os.path.join(out, "prof_" + leg, "**", "*kernel_trace.csv"),
                           recursive=True)
        if not traces:
            continue
        rows = []
        with open(traces[0]) as f:
            for r in csv.DictReader(f):
                if pat not in short_name(r["Kernel_Name"]):
                    continue
                blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                rows.append((int(r["Start_Timestamp"]), short_name(r["Kernel_Name"]), blocks, d))
        if not rows:
            continue
        rows.sort()
        # the full-size launches: the grid the timed region uses (its last)
        g = rows[-1][2]
        full = [x for x in rows if x[2] == g]
        timed = [x[3] for x in full[-k:]]
        rest = [x[3] for x in full[:-k]]
        ts = sorted(timed)
        line = leg_line(out, leg)
        ms = dig(line, path) if line else None
        avg = sum(timed) / len(timed)
        print("| %s | %s | %d | %d | %d | %.2f | %.2f | %.2f | %s | %s | %s |" % (
            leg, full[-1][1], g, len(full), len(timed), avg, ts[len(ts) // 2], ts[0],
            "%.2f" % (sum(rest) / len(rest)) if rest else "--",
            "%.4f" % ms if ms else "--",
            "%.3f" % (avg / 1e3 / ms) if ms else "--"))


def main():
    if len(sys.argv) < 3 or sys.argv[1] not in ("run", "summary"):
        sys.exit(__doc__)
    if sys.argv[1] == "run":
        sys.exit(run(sys.argv[2], sys.argv[3:] or list(LEGS)))
    summary(sys.argv[2])


if __name__ == "__main__":
    main()

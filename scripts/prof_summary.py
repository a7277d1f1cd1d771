#!/usr/bin/env python3
"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace CSV.

    python scripts/prof_summary.py <kernel_trace.csv> > profiles/rNN_kernels.md

rocprofv3 --stats averages every dispatch of a kernel name together; the
bench line launches the EM kernel both at full size (the timed C2 steps)
and at batch sizes 32..4096 (the sweep), so this splits the average by
grid size -- the full-size row is the one bench.py's kernel_ms must match.
"""
import csv
import sys
from collections import defaultdict


def short_name(name):
    """the kernel's name with its template arguments, without the return
    type, the argument list and the namespaces"""
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


def main():
    rows = defaultdict(list)
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "bg::" not in name and not name.startswith("bg_wm_jit"):
                continue  # (bg_wm_jit_*: the run-time compiled WM kernels)
            short = short_name(name)
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            rows[(short, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
                  int(r["VGPR_Count"]), int(r["SGPR_Count"]))].append(d)
    print("| kernel | blocks | VGPR | SGPR | calls | avg us | median us | min us | max us |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (k, g, v, s), ds in sorted(rows.items(), key=lambda x: -sum(x[1])):
        ds.sort()
        print("| %s | %d | %d | %d | %d | %.2f | %.2f | %.2f | %.2f |" % (
            k, g, v, s, len(ds), sum(ds) / len(ds), ds[len(ds) // 2], ds[0], ds[-1]))


if __name__ == "__main__":
    main()

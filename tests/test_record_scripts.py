"""The record tooling: DESIGN.md §6's table comes from a bench line
(scripts/design_table.py) and profiles/rNN_kernels.md from a rocprofv3
kernel trace (scripts/prof_summary.py) -- both checked here on the
committed line §6 names and on kernel names as rocprofv3 prints them."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import prof_summary  # noqa: E402

LINE = os.path.join(ROOT, "profiles", "r04_bench_line.json")


@pytest.mark.parametrize("name,short", [
    ("void bg::(anonymous namespace)::line_slab_kernel<bg::(anonymous namespace)::"
     "HlbFieldsOp<2, 2> >(bg::(anonymous namespace)::HlbFieldsOp<2, 2>::Args, unsigned int)",
     "line_slab_kernel<HlbFieldsOp<2, 2>>"),
    ("void bg::(anonymous namespace)::em_slab_kernel<2, 2, 1>(bg::EmArgs)",
     "em_slab_kernel<2, 2, 1>"),
    ("bg::(anonymous namespace)::dnat_image_kernel(unsigned long const*, unsigned long)",
     "dnat_image_kernel"),
    ("bg_wm_jit_pair", "bg_wm_jit_pair"),
])
def test_kernel_names(name, short):
    assert prof_summary.short_name(name) == short


def test_prof_summary_splits_by_grid(tmp_path):
    trace = tmp_path / "trace.csv"
    rows = [("void bg::(anonymous namespace)::em_slab_kernel<2, 2, 1>(bg::EmArgs)", 512 * 512, 0, 189000),
            ("void bg::(anonymous namespace)::em_slab_kernel<2, 2, 1>(bg::EmArgs)", 512 * 512, 0, 191000),
            ("void bg::(anonymous namespace)::em_slab_kernel<2, 2, 1>(bg::EmArgs)", 512, 0, 4000),
            ("hipMemcpy_kernel", 64, 0, 10)]  # not ours: skipped
    with open(trace, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "VGPR_Count",
                    "SGPR_Count", "Start_Timestamp", "End_Timestamp"])
        for name, grid, t0, t1 in rows:
            w.writerow([name, grid, 512, 28, 80, t0, t1])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_summary.py"),
                          str(trace)], capture_output=True, text=True, check=True).stdout
    lines = out.strip().splitlines()
    assert len(lines) == 4  # header, rule, two grids
    assert lines[2].startswith("| em_slab_kernel<2, 2, 1> | 512 | 28 | 80 | 2 | 190.00 |")
    assert lines[3].startswith("| em_slab_kernel<2, 2, 1> | 1 | 28 | 80 | 1 | 4.00 |")


def design_line():
    """the bench line DESIGN.md §6 says its table was generated from"""
    import re
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        m = re.search(r"generated from one such line \(`([^`]+)`", f.read())
    return os.path.join(ROOT, m.group(1)) if m else LINE


def test_design_table_quotes_the_line():
    line = design_line()
    with open(line) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "design_table.py"), line],
                         capture_output=True, text=True, check=True).stdout
    head = next(l for l in out.splitlines() if l.startswith("| **C2**"))
    assert "%.4f ms" % d["roofline"]["kernel_ms"] in head
    assert "**%.2f**" % d["roofline"]["frac"] in head
    # every row of the table is in DESIGN.md §6 as generated
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        design = f.read()
    for l in out.splitlines():
        if l.startswith("| ") and not l.startswith("|---"):
            assert l in design, l

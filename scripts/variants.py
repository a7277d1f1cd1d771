#!/usr/bin/env python3
"""A/B launch variants of the classify / checksum kernels in ONE process,
interleaved over several rounds (cdna_hip_programming.md §5.4 rule 24).

Variants are selected through the BG_* environment knobs, which only the
measurement build libbessgpu_ab.so reads (`make -C bess_amd/csrc ab`; the
product libbessgpu.so has no knobs and no A/B kernels). Prints one JSON line
per kernel family with median / min milliseconds per launch for each
variant.
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bess_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "scripts", "bin", "libbessgpu_ab.so")
assert _lib.lib().bg_is_ab_build() == 1, "variants.py needs libbessgpu_ab.so"

from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402

KNOBS = ["BG_PPL", "BG_NOLDS", "BG_BLOCKS_PER_CU", "BG_GRID_MULT", "BG_FAT",
         "BG_WM_PHASE", "BG_WM_STREAM",
         "BG_CK_GENERIC", "BG_CK_BLOCKS_PER_CU", "BG_CK_GRID_MULT",
         "BG_CK_TILED", "BG_WM_V", "BG_WM_PF", "BG_EM_PF",
         "BG_NO_SLAB", "BG_SLAB_PF", "BG_WM_BLOCK", "BG_SLAB2", "BG_NAT_PHASE",
         "BG_EM_PAR2", "BG_WM_STREAM_SLOTS", "BG_EM_PAIR", "BG_EM_TG", "BG_NAT_PAR2", "BG_NAT_TW", "BG_LINE_TW", "BG_RW_NT", "BG_WM_LINE", "BG_NAT_OCC", "BG_LINE_OCC", "BG_RW_BPC"]


def set_env(v):
    for k in KNOBS:
        os.environ.pop(k, None)
    for k, x in v.items():
        os.environ[k] = str(x)


def time_variants(fn, variants, rounds=5, reps=40):
    res = {name: [] for name in variants}
    for _ in range(rounds):
        for name, env in variants.items():
            set_env(env)
            fn()  # warm (and re-select the variant)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            b.synchronize()
            res[name].append(a.elapsed_time(b) / reps)
    set_env({})
    return {k: {"median_ms": round(statistics.median(v), 4),
                "min_ms": round(min(v), 4)} for k, v in res.items()}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "em,ck,wm"
    dev = torch.device("cuda:0")
    out = {}
    if "em" in which.split(","):
        n = 16 << 20
        keys, gates, frames = P.em_workload(1000, n)
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        del frames
        g = torch.empty(n, dtype=torch.int16, device=dev)
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
        t.sync(0)
        ref = None
        variants = {
            "default": {}, "slab_pf2": {"BG_SLAB_PF": 2},
            "default_bpc2": {"BG_BLOCKS_PER_CU": 2}, "temporal_gates": {"BG_EM_TG": 1},
            "slab_pf1_bpc1": {"BG_SLAB_PF": 1, "BG_BLOCKS_PER_CU": 1},
            "slab_pf2_bpc1": {"BG_SLAB_PF": 2, "BG_BLOCKS_PER_CU": 1},
            "slab_l2tab_pf2": {"BG_NOLDS": 1, "BG_SLAB_PF": 2},
            "lane": {"BG_NO_SLAB": 1},
            "slab2_512": {"BG_SLAB2": 512},
            "slab2_1024": {"BG_SLAB2": 1024},
            "slab2_1024_l2tab": {"BG_SLAB2": 1024, "BG_NOLDS": 1},
        }
        # every variant must give identical gates
        for name, env in variants.items():
            set_env(env)
            t.classify(d, 64, n, 8192, g)
            torch.cuda.synchronize()
            if ref is None:
                ref = g.clone()
            assert torch.equal(g, ref), name
        r = time_variants(lambda: t.classify(d, 64, n, 8192, g), variants)
        for k in r:
            r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
            r[k]["GBps_66B"] = round(66 * n / (r[k]["median_ms"] * 1e-3) / 1e9, 1)
        out["em"] = r
        del d, g
    if "em1500" in which:
        # bench.py's EM_1500B leg: 1 K-rule 5-tuple ExactMatch over 4 M
        # 1496 B frames in 2 KB slots (first 64 B written): pair loads
        # (em_pair_kernel) vs one lane per packet (em_classify_kernel)
        n = 1 << 22
        keys, gates, hdr = P.em_workload(1000, n, seed=0x5EED, stride=64,
                                         frame_len=1496, pkt_seed=0x1500)
        d = torch.zeros(n * 2048, dtype=torch.uint8, device=dev)
        d.view(n, 2048)[:, :64] = torch.from_numpy(hdr).to(dev)
        del hdr
        g = torch.empty(n, dtype=torch.int16, device=dev)
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
        t.sync(0)
        variants = {"pair": {}, "lane": {"BG_EM_PAIR": 0}}
        ref = None
        for name, env in variants.items():
            set_env(env)
            t.classify(d, 2048, n, 8192, g)
            torch.cuda.synchronize()
            if ref is None:
                ref = g.clone()
            assert torch.equal(g, ref), name
        r = time_variants(lambda: t.classify(d, 2048, n, 8192, g), variants, reps=20)
        for k in r:
            r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
        out["em1500"] = r
        del d, g
    if "c5" in which:
        n = 16 << 20
        keys, gates, frames = P.em_workload(1 << 20, n)
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        del frames
        g = torch.empty(n, dtype=torch.int16, device=dev)
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
        t.sync(0)
        variants = {
            "default": {}, "both_tags": {"BG_EM_PAR2": 1}, "slab_pf2": {"BG_SLAB_PF": 2},
            "slab_bpc3": {"BG_BLOCKS_PER_CU": 3},
            "slab_pf0": {"BG_SLAB_PF": 0},
            "slab_bpc2": {"BG_BLOCKS_PER_CU": 2},
            "slab_bpc4": {"BG_BLOCKS_PER_CU": 4},
            "lane_p1": {"BG_NO_SLAB": 1, "BG_PPL": 1},
            "lane_p2": {"BG_NO_SLAB": 1, "BG_PPL": 2},
            "lane_p2_x2": {"BG_NO_SLAB": 1, "BG_PPL": 2, "BG_GRID_MULT": 2},
            "lane_pf": {"BG_NO_SLAB": 1, "BG_EM_PF": 1},
        }
        ref = None
        for name, env in variants.items():
            set_env(env)
            t.classify(d, 64, n, 8192, g)
            torch.cuda.synchronize()
            if ref is None:
                ref = g.clone()
            assert torch.equal(g, ref), name
        r = time_variants(lambda: t.classify(d, 64, n, 8192, g), variants,
                          reps=10)
        for k in r:
            r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
        out["c5"] = r
        del d, g
    if "ck" in which:
        n = 1 << 20
        frames = P.cksum_workload(n, frame_len=1496)
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        l4 = torch.empty(n, dtype=torch.int16, device=dev)
        variants = {"words_d1": {}, "reload_d2": {"BG_CK_TILED": 9},
                    "generic": {"BG_CK_GENERIC": 1},
                    "regs_d1": {"BG_CK_TILED": 1}, "reload_d1": {"BG_CK_TILED": 2},
                    "reload_d3": {"BG_CK_TILED": 3}, "regs_d2": {"BG_CK_TILED": 4},
                    "w5_d2": {"BG_CK_TILED": 5}, "w5_d3": {"BG_CK_TILED": 6},
                    "stash_d2": {"BG_CK_TILED": 7}, "words_d2": {"BG_CK_TILED": 8},
                    "words_d1_w5": {"BG_CK_TILED": 10},
                    "words_nt": {"BG_CK_TILED": 14},
                    "words_d1_x8": {"BG_CK_GRID_MULT": 8},
                    "words_d1_x2": {"BG_CK_GRID_MULT": 2}}
        outs = {}
        for name, env in variants.items():
            dd = torch.from_numpy(frames.reshape(-1)).to(dev)
            set_env(env)
            F.cksum(dd, 2048, n, 3, False, None, l4)
            torch.cuda.synchronize()
            outs[name] = (dd.cpu(), l4.cpu())
        base = next(iter(outs.values()))
        for name, (x, y) in outs.items():
            assert torch.equal(x, base[0]) and torch.equal(y, base[1]), name
        del outs
        # (idempotent after the first pass: recompute writes the same bytes)
        r = time_variants(lambda: F.cksum(d, 2048, n, 3, False, None, l4),
                          variants)
        for k in r:
            r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
            r[k]["GBps_1502B"] = round(1502 * n / (r[k]["median_ms"] * 1e-3) / 1e9, 1)
        out["ck"] = r
        del d
    if "natphase" in which:
        # NAT established flows as bench.py times them (16 M packets of 64 K
        # flows, fresh copies, `now` advancing): everything vs. without the
        # forward timestamp read and refresh (BG_NAT_PHASE=1) vs. without
        # the table lookup (2)
        from bess_amd.modules import NAT
        nflow, n = 1 << 16, 1 << 24
        _, _, flows = P.em_workload(16, nflow, seed=0x5EED, pkt_seed=17)
        zero = (flows[:, 34] == 0) & (flows[:, 35] == 0)
        flows[zero, 35] = 1
        rng = np.random.default_rng(17)
        slab = flows[rng.integers(0, nflow, n)]
        m = NAT(ext_addrs=[{"ext_addr": "100.64.0.1"}, {"ext_addr": "100.64.0.2"}],
                seed=0x5EED)
        t0 = 10 ** 12
        g = torch.empty(n, dtype=torch.int16, device=dev)
        m.process_device(torch.from_numpy(flows.reshape(-1).copy()).to(dev), 64, nflow, g, t0)
        src = torch.from_numpy(slab.reshape(-1)).to(dev)
        now = [t0]
        phases = (("full", {}), ("no_timestamp", {"BG_NAT_PHASE": 1}),
                  ("no_lookup", {"BG_NAT_PHASE": 2}), ("both_tags", {"BG_NAT_PAR2": 1}),
                  ("temporal_lines", {"BG_NAT_TW": 1}), ("occ2", {"BG_NAT_OCC": 2}),
                  ("occ3", {"BG_NAT_OCC": 3}))
        res = {name: [] for name, _ in phases}
        for _ in range(3):
            for name, env in phases:
                set_env(env)
                copies = [src.clone() for _ in range(8)]
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for c in copies:
                    now[0] += 1
                    m.process_device(c, 64, n, g, now[0])
                b.record()
                b.synchronize()
                res[name].append(a.elapsed_time(b) / len(copies))
                del copies
        set_env({})
        out["natphase"] = {k: {"median_ms": round(statistics.median(v), 4),
                               "min_ms": round(min(v), 4)} for k, v in res.items()}
    if "wmphase" in which:
        # C4 on the dense header slab, timed up to each phase of
        # wm_tags_kernel (BG_WM_PHASE: 1 header read + key, 2 + the 8
        # tuple hashes, tag reads and queue writes, 3 everything but the
        # checks' L2 loads, 0 everything)
        n = 1 << 23
        rk, rm, prio, gates, frames, _ = P.wm_workload(100000, 1 << 20, stride=64,
                                                      sizes=((60, 1),))
        d = torch.from_numpy(frames.reshape(-1)).to(dev).repeat(8)
        g = torch.empty(n, dtype=torch.int16, device=dev)
        t = F.WmTable(P.FIVE_TUPLE)
        for k, m, p, gg in zip(rk, rm, prio, gates):
            t.add(k.tobytes(), m.tobytes(), int(p), int(gg))
        t.sync(0)
        variants = {"full": {}, "read_key": {"BG_WM_PHASE": 1},
                    "enqueue": {"BG_WM_PHASE": 2},
                    "checks_no_l2": {"BG_WM_PHASE": 3}}
        # the streamed form (producer waves) and the one without
        variants.update({k + "_stream": dict(v, BG_WM_STREAM=1)
                         for k, v in list(variants.items())})
        r = time_variants(lambda: t.classify(d, 64, n, 8192, g), variants,
                          reps=20)
        for k in r:
            r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
        out["wmphase"] = r
        # the same on the frames in 2 KB slots (1 M of them)
        f2 = torch.from_numpy(P.wm_workload(100000, 1 << 20, stride=2048)[4].reshape(-1)).to(dev)
        n2 = 1 << 20
        r = time_variants(lambda: t.classify(f2, 2048, n2, 8192, g), variants, reps=20)
        for k in r:
            r[k]["Mpps"] = round(n2 / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
        out["wmphase_2k"] = r
        del d, g, f2
    if "rewrite" in which:
        # bench.py's Rewrite leg: 16 M packets in 192 B slots, 4 templates
        # of 60 B; normal vs streaming stores (BG_RW_NT)
        from bess_amd.modules import Rewrite
        n = 16 << 20
        m = Rewrite(templates=[bytes([i]) * 60 for i in range(1, 5)])
        d = torch.zeros(n * 192, dtype=torch.uint8, device=dev)
        dh = torch.empty(n, dtype=torch.int16, device=dev)
        dl = torch.empty(n, dtype=torch.int32, device=dev)
        r = time_variants(lambda: m.process_device(d, 192, n, dh, dl),
                          {"stores": {}, "stores_nt": {"BG_RW_NT": 1},
                           "bpc2": {"BG_RW_BPC": 2}, "bpc4": {"BG_RW_BPC": 4},
                           "bpc16": {"BG_RW_BPC": 16}}, reps=10)
        out["rewrite"] = r
        del d
    if "lineocc" in which:
        # the read-only line ops (HashLB l4 and 5-tuple fields on 16 M 64 B
        # packets) at the occupancy limit vs 2 / 3 workgroups per CU
        from bess_amd.modules import HashLB
        n = 16 << 20
        _, _, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=5)
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        g = torch.empty(n, dtype=torch.int16, device=dev)
        five = [{"offset": o, "num_bytes": sz} for o, sz in P.FIVE_TUPLE]
        for name, kw in (("hashlb_l4", dict(mode="l4")), ("hashlb_fields", dict(fields=five))):
            m = HashLB(gates=list(range(8)), **kw)
            out["lineocc_" + name] = time_variants(
                lambda: m.process_device(d, 64, n, g),
                {"default": {}, "occ2": {"BG_LINE_OCC": 2}, "occ3": {"BG_LINE_OCC": 3}}, reps=20)
        del d
    if "linew" in which:
        # the writing header-line ops (UpdateTTL, StaticNAT: 16 M 64 B
        # packets in place, as bench.py) with their written-back lines
        # stored nontemporally (the default) vs normally (BG_LINE_TW); TTL starts at 200
        # and the 180 launches here stay above 1
        from bess_amd.modules import StaticNAT, UpdateTTL
        n = 16 << 20
        _, _, frames = P.em_workload(1000, n, seed=0x5EED, pkt_seed=11)
        frames[:, 22] = 200
        rng = np.random.default_rng(13)
        hit = rng.random(n) < 0.5
        frames[hit, 26] = 10
        frames[hit, 27] = rng.integers(0, 8, int(hit.sum()), dtype=np.uint8)
        g = torch.empty(n, dtype=torch.int16, device=dev)
        pairs = []  # bench.py nat_pairs(): 10.i/16 <-> 100.i/16, both ways
        for back in (0, 1):
            for i in range(8):
                a, b = ("100.%d" % i, "10.%d" % i) if back else ("10.%d" % i, "100.%d" % i)
                pairs.append({"int_range": {"start": a + ".0.0", "end": a + ".255.255"},
                              "ext_range": {"start": b + ".0.0", "end": b + ".255.255"}})
        for name, m in (("ttl", UpdateTTL()), ("static_nat", StaticNAT(pairs=pairs))):
            d = torch.from_numpy(frames.reshape(-1)).to(dev)
            r = time_variants(lambda: m.process_device(d, 64, n, g),
                              {"lines_nt": {}, "lines": {"BG_LINE_TW": 1},
                               "occ2": {"BG_LINE_OCC": 2}, "occ3": {"BG_LINE_OCC": 3}},
                              reps=8)
            out["linew_" + name] = r
            del d
    if "wmdirect" in which:
        # C4 with the source-port tuple direct (the round-4 policy: every
        # two-byte tuple, BG_WM_DIRECT2_MIN=0) vs hashed (>= 32768 rules);
        # each table built under its setting; header slab and 2 KB slots
        rk, rm, prio, gates, frames, _ = P.wm_workload(100000, 1 << 20, stride=64,
                                                      sizes=((60, 1),))
        f2 = torch.from_numpy(P.wm_workload(100000, 1 << 20, stride=2048)[4]
                              .reshape(-1)).to(dev)
        d = torch.from_numpy(frames.reshape(-1)).to(dev).repeat(8)
        res = {}
        ref = {}
        for name, env in (("sport_hashed", {}), ("sport_direct", {"BG_WM_DIRECT2_MIN": 0})):
            set_env(env)
            os.environ.pop("BG_WM_DIRECT2_MIN", None)
            os.environ.update({k: str(v) for k, v in env.items()})
            t = F.WmTable(P.FIVE_TUPLE)
            for k, m, p, gg in zip(rk, rm, prio, gates):
                t.add(k.tobytes(), m.tobytes(), int(p), int(gg))
            t.sync(0)
            t.jit_wait()  # (time the run-time compiled kernel of this shape)
            os.environ.pop("BG_WM_DIRECT2_MIN", None)
            r = {"direct_tuples": t.direct_tuples()}
            for lay, dd, stride, n in (("slab", d, 64, 1 << 23), ("2k", f2, 2048, 1 << 20)):
                g = torch.empty(n, dtype=torch.int16, device=dev)
                t.classify(dd, stride, n, 8192, g)
                torch.cuda.synchronize()
                if lay in ref:
                    r[lay + "_same_gates"] = bool(torch.equal(g, ref[lay]))
                else:
                    ref[lay] = g.clone()
                tt = time_variants(lambda: t.classify(dd, stride, n, 8192, g), {"x": {}},
                                   reps=20)["x"]
                r[lay] = tt
            res[name] = r
            del t
        out["wmdirect"] = res
        del d, f2
    if "wmstream" in which:
        # C4 (ahead-of-time kernel): every wave loading its own windows vs
        # the streamed form at its deep producer depth (the ring C4's tag
        # words leave) and at the shallow one (ring capped at 28 slots);
        # header slab (8 M packets) and 2 KB slots (1 M); gates compared
        rk, rm, prio, gates, frames, _ = P.wm_workload(100000, 1 << 20, stride=64,
                                                      sizes=((60, 1),))
        t = F.WmTable(P.FIVE_TUPLE)
        for k, m, p, gg in zip(rk, rm, prio, gates):
            t.add(k.tobytes(), m.tobytes(), int(p), int(gg))
        t.sync(0)
        variants = {"per_wave": {}, "per_wave_line": {"BG_WM_LINE": 1},
                    "stream_deep": {"BG_WM_STREAM": 1},
                    "stream_d16": {"BG_WM_STREAM": 1, "BG_WM_STREAM_SLOTS": 28}}
        layouts = (("slab", torch.from_numpy(frames.reshape(-1)).to(dev).repeat(8), 64, 1 << 23),
                   ("2k", torch.from_numpy(P.wm_workload(100000, 1 << 20, stride=2048)[4]
                                           .reshape(-1)).to(dev), 2048, 1 << 20))
        for name, d, stride, n in layouts:
            g = torch.empty(n, dtype=torch.int16, device=dev)
            ref = None
            same = {}
            for v, env in variants.items():
                set_env(env)
                g.fill_(0)
                t.classify(d, stride, n, 8192, g)
                torch.cuda.synchronize()
                if ref is None:
                    ref = g.clone()
                same[v] = bool(torch.equal(g, ref))
            r = time_variants(lambda: t.classify(d, stride, n, 8192, g), variants, reps=20)
            for k in r:
                r[k]["Mpps"] = round(n / (r[k]["median_ms"] * 1e-3) / 1e6, 1)
                r[k]["same_gates"] = same[k]
            out["wmstream_" + name] = r
            del d, g
    if "wm" in which.split(","):
        n = 1 << 22
        rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n, stride=64,
                                                      sizes=((60, 1),))
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        g = torch.empty(n, dtype=torch.int16, device=dev)
        tables = {}
        for kb in (0, 32, 64, 128):  # key filter size is fixed at sync time
            os.environ["BG_WM_FILTER_KB"] = str(kb)
            t = F.WmTable(P.FIVE_TUPLE)
            for k, m, p, gg in zip(rk, rm, prio, gates):
                t.add(k.tobytes(), m.tobytes(), int(p), int(gg))
            t.sync(0)
            tables[kb] = t
        os.environ.pop("BG_WM_FILTER_KB", None)
        variants = {"default": (64, {}),
                    "seq_pf": (64, {"BG_WM_V": 1, "BG_WM_PF": 1, "BG_PPL": 1}),
                    "seq_p2": (64, {"BG_WM_V": 1, "BG_PPL": 2}),
                    "seq_pf_f128": (128, {"BG_WM_V": 1, "BG_WM_PF": 1, "BG_PPL": 1}),
                    "nofilter_seq_pf": (0, {"BG_WM_V": 1, "BG_WM_PF": 1, "BG_PPL": 1}),
                    "k1024": (64, {"BG_WM_BLOCK": 1024}),
                    "k1024_p2": (64, {"BG_WM_BLOCK": 1024, "BG_PPL": 2}),
                    "k1024_f128": (128, {"BG_WM_BLOCK": 1024}),
                    "k1024_f32": (32, {"BG_WM_BLOCK": 1024}),
                    "nofilter_default": (0, {})}
        ref = None
        for name, (kb, env) in variants.items():
            set_env(env)
            tables[kb].classify(d, 64, n, 8192, g)
            torch.cuda.synchronize()
            if ref is None:
                ref = g.clone()
            assert torch.equal(g, ref), name
        res = {k: [] for k in variants}
        for _ in range(5):
            for name, (kb, env) in variants.items():
                set_env(env)
                tables[kb].classify(d, 64, n, 8192, g)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    tables[kb].classify(d, 64, n, 8192, g)
                b.record()
                b.synchronize()
                res[name].append(a.elapsed_time(b) / 20)
        set_env({})
        r = {}
        for k, v in res.items():
            med = statistics.median(v)
            r[k] = {"median_ms": round(med, 4), "min_ms": round(min(v), 4),
                    "Mpps": round(n / (med * 1e-3) / 1e6, 1),
                    "table": tables[variants[k][0]].table_info()}
        out["wm"] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""bench.py -- device-resident parse+match throughput on MI355X.

Headline (BASELINE.json metric "Mpps + %HBM-roofline, device-resident
parse+match, 64B/1500B, 1/2/4/8 GPU"): config C2 -- 64 B packets (60 B
frames), 1K-rule 5-tuple ExactMatch, 16 M packets resident in HBM per GPU.
One step = one pass of the hot path (ExactMatch::ProcessBatch semantics:
header-field extract + hash -> flow-table match -> egress gate) over the
resident slab.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rules R]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

`--gpus N` without torchrun starts the N ranks itself (torch.distributed.run
as a child process, before anything touches a GPU) and exits with its code;
under torchrun WORLD_SIZE must equal N.

N > 1: every rank owns its own 16 M packets (weak scaling, no data-path
collective). The headline stays C2 at every N so the driver's per-N values
compare like with like. The line also carries C5 at that N: 1 M rules
sharded over the N GPUs -- rank r inserts only partition r's rules, the
ranks agree on the layout with an all-reduce, build their partition, and
one RCCL all-gather over xGMI assembles the replicated table on every GPU
(the only collective; control path, timed separately) -- then every rank
classifies its own 16 M packets through the gathered 1 M-rule table.

Rank 0 prints ONE JSON line. Secondary configs (C1 CPU plumbing, C3
checksum, C4 wildcard, the §8f modules, batch-size sweeps, host legs) are
measured at N = 1 only, as extra keys.
"""
import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table
EM_BYTES_PER_PKT = 66  # 64 B header line read + 2 B gate written
CK_BYTES_PER_PKT = 1502  # 1496 B frame read + IP csum + L4 csum + gate (2 B each)
PCIE_GBS = 63.0  # host link, PCIe Gen5 x16 per direction (MI355X_MICROARCH.md, spec)


def pcie(mpps, h2d, d2h):
    """A host-memory leg against its link: bytes per packet each way (the
    staged window or the in-place frame reads host -> device, gates and
    written-back lines device -> host), their GB/s at `mpps`, and the busier
    direction's fraction of the spec rate (the host legs' bound)"""
    if not isinstance(mpps, (int, float)):
        return None
    gh, gd = mpps * 1e6 * h2d / 1e9, mpps * 1e6 * d2h / 1e9
    return {"h2d_bytes_per_pkt": h2d, "d2h_bytes_per_pkt": d2h,
            "h2d_GBps": round(gh, 2), "d2h_GBps": round(gd, 2),
            "pcie_frac": round(max(gh, gd) / PCIE_GBS, 4)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--rules", type=int, default=1000)
    ap.add_argument("--pkts", type=int, default=16 << 20)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the C3/C4/sweep secondary measurements")
    ap.add_argument("--no-cpu", action="store_true", help="skip cpu_baseline")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host end-to-end legs (16 launching threads "
                         "crash rocprofv3's kernel tracer)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--diag", action="store_true",
                    help="host-leg diagnostics (pipe counters, cycles) to stderr")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed device work before each leg's warm-up "
                         "(clock_settle); 0 = none")
    ap.add_argument("--cpu-table-only", action="store_true",
                    help="no GPU: the N-rank sharded table build of C5 over "
                         "gloo (CPU tests of the multi-GPU launch and control "
                         "path); prints the line with value null")
    ap.add_argument("--pipe-threads", default="1,4,16",
                    help="worker threads of the bg_pipe legs")
    ap.add_argument("--wm-layout", default="both", choices=("both", "slab", "2k"),
                    help="C4 layouts to time (PMC passes time one at a time)")
    ap.add_argument("--em1500-pkts", type=int, default=1 << 22,
                    help="resident 1500 B packets of the EM 1500 B leg (2 KB slots)")
    ap.add_argument("--c5-rules", type=int, default=1 << 20,
                    help="rules of the sharded C5 table in the N > 1 line")
    ap.add_argument("--no-churn", action="store_true",
                    help="NAT: skip the new-flow batch stream (PMC passes)")
    ap.add_argument("--lib", default="",
                    help="time another build of libbessgpu.so (same-box A/B)")
    ap.add_argument("--drive", default="",
                    help="another build of tests/bessd_shell's driver (same-box A/B)")
    ap.add_argument("--only", default="", help="c1|cksum|em1500|wm|c5|hashlb|acl|iplookup|ttl|nat|dnat|rewrite|pipe|plugin|sweep (profiling runs)")
    return ap.parse_args()


class Timer:
    """HIP events on the stream the kernels are launched on (torch's current
    stream: libbessgpu launches on the hipStream_t we pass, which is it)."""

    def __init__(self, torch):
        self.torch = torch
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def start(self):
        self.a.record()

    def stop_ms(self):
        self.b.record()
        self.b.synchronize()
        return self.a.elapsed_time(self.b)


def load_traffic(key):
    """HBM bytes per launch of the workload's kernel, measured with
    rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, gfx950-corrected) and
    written by scripts/pmc_traffic.py to profiles/rNN_traffic.json; the
    latest round's file is used."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            e = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    return None if e is None else e.get("traffic_bytes")


def shape_ceiling(shape, pkts, ms):
    """The measured ceiling of an access shape (scripts/hbm_probe.hip, the
    latest profiles/r*_calibration.json): the probe's packet rate, the time
    it would take for `pkts`, and this kernel's fraction of it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_calibration.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            e = json.load(f)["shapes"][shape]["ceiling"]
    except (OSError, ValueError, KeyError):
        return None
    floor_ms = pkts / (e["Gpkts_per_s"] * 1e9) * 1e3
    return {"shape": shape, "probe_Gpkts_per_s": e["Gpkts_per_s"],
            "probe_ms_for_these_pkts": round(floor_ms, 4),
            "frac_of_ceiling": round(floor_ms / ms, 4),
            "source": os.path.relpath(files[-1], ROOT)}


def placed_slab(make, probe, torch, candidates=3):
    """A resident slab for a scattered-read leg (a 32 B window per 2 KB
    slot: C4 on 2 KB slots, ExactMatch on 1500 B frames) whose placement
    does not slow it down. Such a read runs 0.188 ms on most 16 GB
    allocations and 0.203 / 0.220 ms on about one in three, the same bytes
    in the same process: the physical pages the allocation gets decide it
    (profiles/r06/placement_*.json; not the address alignment,
    the allocation flags or the TLB). `make()` builds a candidate slab,
    `probe(slab)` times the leg's own launch on it (ms): `candidates` are
    built and probed, the fastest is kept, the others are freed, and every
    candidate's probe time goes into the line."""
    times, best, best_ms = [], None, None
    for _ in range(candidates):
        sl = make()
        ms = probe(sl)
        times.append(round(ms, 4))
        if best is None or ms < best_ms:
            best, best_ms = sl, ms
        else:
            del sl
        torch.cuda.empty_cache()
    return best, {"candidates_probe_ms": times, "kept": times.index(round(best_ms, 4)),
                  "why": "scattered 2 KB-slot reads depend on the slab's physical pages "
                         "(DESIGN section 8): the fastest of the candidate allocations is kept"}


def probe_ms(step, torch, k=10):
    """ms per launch of `step` over k launches after one, HIP events"""
    step()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        step()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / k


def traffic_gbs(key, kernel_ms):
    """PMC bytes per launch / measured launch duration, in GB/s (same basis
    as roofline.achieved); None until profiles/ holds a PMC measurement."""
    b = load_traffic(key)
    return None if b is None else round(b / (kernel_ms * 1e-3) / 1e9, 1)


def em_setup(args, rank, world, dev, torch, dist):
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    t0 = time.time()
    # same rule set on every rank, rank-specific packets
    keys, gates, frames = P.em_workload(args.rules, args.pkts, seed=0x5EED,
                                        pkt_seed=0x5EED + 7919 * rank)
    log("[rank %d] workload generated in %.1fs" % (rank, time.time() - t0))
    d_frames = torch.from_numpy(frames.reshape(-1)).to(dev)
    del frames
    d_gates = torch.empty(args.pkts, dtype=torch.int16, device=dev)
    t = F.EmTable(P.em_fields_5tuple())
    t0 = time.time()
    # C2's 1K rules: every rank builds the whole (38 KB) table itself; the
    # all-gather is C5's (run_c5_multi)
    t.add_many(keys, gates)
    log("[rank %d] %d rules inserted in %.1fs" % (rank, len(t), time.time() - t0))
    table = {"rules": len(keys), "build": "replicated (each GPU builds the rule set)"}
    t.sync(dev.index)
    nbytes, in_lds = t.table_info()
    table.update({"bytes": nbytes, "in_lds": in_lds})
    return t, d_frames, d_gates, keys, gates, table


def em_parity_sample(t, d_frames, d_gates, keys, gates, n, torch):
    """Bit-exact check of the first n packets against the CPU oracle."""
    from bess_amd import packets as P
    from oracle import oracle as O
    import ctypes as C
    frames = d_frames[:n * 64].cpu().numpy()
    got = d_gates[:n].cpu().numpy().view(np.uint16)
    L = O.lib()
    em = oracle_em_bulk(keys, gates)
    want = np.zeros(n, np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, n, 8192, want.ctypes.data)
    L.or_em_free(em)
    return bool((got == want).all())


def cpu_info():
    """The host CPUs a CPU baseline may use: every CPU of the affinity mask
    within the lease's CPU share (the GPU pool sets OMP_NUM_THREADS to the
    CPUs it grants one GPU's job; nproc reports the whole machine). Returns
    (threads, record for the JSON line)."""
    aff = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    share = int(share) if share and share.isdigit() and int(share) > 0 else aff
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads = max(1, min(aff, share))
    return threads, {"nproc": os.cpu_count(), "affinity_cpus": aff,
                     "lease_cpu_share": share, "cpu_model": model}


def cpu_baseline(res, threads, sample, kind="port", unit="Mpps"):
    """cpu_baseline object: `res` {threads: rate} at 1 and T threads"""
    _, info = cpu_info()
    out = {"value": round(res[threads], 2), "unit": unit, "cores": threads,
           "kind": kind, "single_core_mpps": round(res[1], 2), "sample": sample}
    out.update(info)
    return out


def cpu_rate(bench, n, seconds, threads=None, max_reps=None):
    """Time the oracle's pthread bench driver `bench(nthreads, reps)` (returns
    seconds) at 1 thread and at T threads (default: every CPU the lease
    grants, cpu_info); about `seconds` of CPU work in total. Returns
    (T, {threads: Mpps})."""
    if threads is None:
        threads, _ = cpu_info()
    res = {}
    for nt in sorted({1, threads}):
        t1 = bench(nt, 1)
        reps = max(1, int(seconds / 2 / max(t1, 1e-6)))
        if max_reps:
            reps = min(reps, max_reps)
        res[nt] = n * reps / bench(nt, reps) / 1e6
    return threads, res


def cpu_baseline_em(keys, gates, seconds):
    """The oracle (plain-C restatement of ExactMatch::ProcessBatch with a
    CuckooMap/CRC32C table, 32-packet batches) timed on this host's cores
    over packets laid out like BESS snbufs (2624 B stride, frame at +512)."""
    from bess_amd import packets as P
    from oracle import oracle as O
    import ctypes as C
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    sizes = [s for _, s in P.FIVE_TUPLE]
    pos = np.cumsum([0] + sizes)
    ptrs = (C.c_void_p * 5)()
    lens = (C.c_size_t * 5)(*sizes)
    for k, g in zip(np.ascontiguousarray(keys), gates):
        for j in range(5):
            ptrs[j] = k.ctypes.data + int(pos[j])
        L.or_em_add_rule(em, int(g), ptrs, lens, 5, None, 0)
    n = 1 << 18
    _, _, frames = P.em_workload(len(keys), n, seed=0x5EED, pkt_seed=77)
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 64] = frames
    base = snb.ctypes.data + 512
    out = np.zeros(n, np.uint16)
    threads, res = cpu_rate(
        lambda nt, reps: L.or_em_bench(em, base, 2624, n, 8192, out.ctypes.data,
                                       nt, reps), n, seconds)
    L.or_em_free(em)
    return cpu_baseline(res, threads,
                        "%d 64B pkts x reps, 1K-rule 5-tuple ExactMatch, snbuf "
                        "layout (2624 B stride), 32-pkt batches, %d pinned "
                        "threads" % (n, threads))


def run_em(args, rank, world, dev, torch, dist):
    from bess_amd import flowtable as F  # noqa: F401
    t, d_frames, d_gates, keys, gates, table = em_setup(args, rank, world, dev,
                                                       torch, dist)
    n = args.pkts

    def step():
        t.classify(d_frames, 64, n, 8192, d_gates)

    # parity first: the host-side check leaves the GPU idle for seconds,
    # so the warmup that follows brings the clocks back up before timing
    step()
    torch.cuda.synchronize()
    parity = em_parity_sample(t, d_frames, d_gates, keys, gates,
                              min(n, 1 << 20), torch)
    # settle with the headline's own (idempotent) launch: after ~5 launches
    # the next ~45 run 10-15 % slow whatever the slab's history, then the
    # kernel holds its steady state (a power-management transient, launch by
    # launch: profiles/r06/first_launch_r06v.json); the driver's --warmup 5
    # would otherwise time that transient (0.170-0.176 against 0.164 ms for
    # 200 steps on one box, profiles/r06/headline_steps_r06u.json)
    clock_settle(args, torch, step)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timer = Timer(torch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    timer.start()
    for _ in range(args.steps):
        step()
    kern_ms = timer.stop_ms()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - w0
    if world > 1:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms = tt.tolist()
        ok = torch.tensor([1 if parity else 0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        parity = bool(ok.item())
    return {"t": t, "d_frames": d_frames, "d_gates": d_gates, "keys": keys,
            "gates": gates, "wall": wall, "kern_ms": kern_ms, "n": n,
            "parity": parity, "table": table}


def em_sweep(r, torch, batches=(32, 64, 128, 256, 512, 1024, 2048, 4096)):
    """Per-launch batch-size sweep (SURVEY C2 'batch 32->4096'): each batch
    of B packets is one kernel launch, 512 batches per measurement.
      stream: back-to-back bg_em_classify calls on one stream (host launch
              cost included: what one BESS worker issuing B-packet batches
              sees; the stream attached with bg_stream_attach);
      graph:  the 512 launches captured in a HIP graph and replayed (no
              host cost; the runtime may overlap independent launches);
      persistent: ONE running kernel (bg_ring) drains the batches as host
              threads submit their descriptors, each on its own submission
              lane (bg_ring_run: the 16M-packet slab in B-packet batches
              split over 1, 4 or 16 submitter threads, each thread 4 passes
              over its part; wall time from the threads' start to the last
              batch's completion, per pass; no HIP graph)."""
    from bess_amd import flowtable as F
    t, d_frames, d_gates = r["t"], r["d_frames"], r["d_gates"]
    out = {"stream": {}, "graph": {}, "persistent": {}}
    s = torch.cuda.Stream()
    nl = 512

    import ctypes as C
    from bess_amd import lib
    classify = lib().bg_em_classify
    fp, gp, sp = d_frames.data_ptr(), d_gates.data_ptr(), C.c_void_p(s.cuda_stream)
    # the worker's stream attached (bg_stream_attach): a rule change fences it
    # once, instead of an event recorded per launch; detached below
    if lib().bg_stream_attach(sp):
        raise RuntimeError("bg_stream_attach failed")

    def launches(B):  # straight C-ABI calls: no per-launch tensor slicing
        for j in range(nl):
            off = j * B
            rc = classify(t.h, C.c_void_p(fp + off * 64), 64, B, 8192,
                          C.c_void_p(gp + off * 2), sp)
            if rc:
                raise RuntimeError("bg_em_classify failed: %d" % rc)

    def timed(fn, reps=5):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        b.synchronize()
        return a.elapsed_time(b) / reps

    for B in batches:
        with torch.cuda.stream(s):
            launches(B)
            torch.cuda.synchronize()
            ms = timed(lambda: launches(B))
        out["stream"][str(B)] = round(nl * B / (ms * 1e-3) / 1e6, 1)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                launches(B)
        g.replay()
        torch.cuda.synchronize()
        ms = timed(g.replay)
        out["graph"][str(B)] = round(nl * B / (ms * 1e-3) / 1e6, 1)
    lib().bg_stream_detach(sp)
    npk = min(16 << 20, r["n"])  # the C2 slab: enough tickets at any batch size
    launches0 = 0
    for T in (1, 4, 16):  # a ring with one submission lane per submitter
        ring = F.Ring(t, slots=4096, lanes=T)
        ring.set_coherence(1, 0)  # as the pipes use it (ExactMatch module)
        key = "persistent" if T == 1 else "persistent_%dsub" % T
        out[key] = {}
        for B in batches:
            ring.run_lanes(d_frames, 64, npk, B, 8192, d_gates, T)  # warm
            best = min(ring.run_lanes(d_frames, 64, npk, B, 8192, d_gates, T, reps=4)
                       for _ in range(3))
            out[key][str(B)] = round(npk / best / 1e6, 1)
        launches, blocks = ring.info()
        launches0 += launches
        ring.close()
    out["persistent_info"] = {"packets_per_point": npk, "kernel_launches": launches0,
                              "workgroups": blocks, "slots_per_lane": 4096,
                              "lanes": "one per submitter", "submitters": [1, 4, 16],
                              "timing": "host wall of 4 passes per thread / 4, best of 3"}
    return out


def run_cksum(args, dev, torch):
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    n = 1 << 20
    frames = P.cksum_workload(n, frame_len=1496, stride=2048)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    ref = frames[:4096].copy()
    cpu_frames = frames[:1 << 16].copy()
    del frames
    l4g = torch.empty(n, dtype=torch.int16, device=dev)
    F.cksum(d, 2048, n, 3, False, None, l4g)
    torch.cuda.synchronize()
    # parity on a sample: oracle on the original frames vs device result
    from oracle import oracle as O
    ipw, l4w = O.cksum_process(ref, 2048, 4096, 3, False)
    got = d[:4096 * 2048].cpu().numpy().reshape(4096, 2048)
    parity = bool((got == ref).all() and
                  (l4g[:4096].cpu().numpy().view(np.uint16) == l4w).all())
    clock_settle(args, torch, lambda: F.cksum(d, 2048, n, 3, False, None, l4g))
    for _ in range(args.warmup):  # recompute is idempotent
        F.cksum(d, 2048, n, 3, False, None, l4g)
    torch.cuda.synchronize()
    timer = Timer(torch)
    torch.cuda.synchronize()
    k = leg_steps(args)
    timer.start()
    for _ in range(k):
        F.cksum(d, 2048, n, 3, False, None, l4g)
    ms = timer.stop_ms() / k
    mpps = n / (ms * 1e-3) / 1e6
    gbs = CK_BYTES_PER_PKT * n / (ms * 1e-3) / 1e9
    out = {"workload": "C3: 1500B pkts (1496B frames, 2048B slots), "
                       "IPChecksum->L4Checksum recompute, 50/50 UDP/TCP",
           "pkts": n, "ms_per_step": round(ms, 4), "Mpps": round(mpps, 1),
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "traffic": traffic_gbs("cksum", ms),
                        "traffic_bytes_per_launch": load_traffic("cksum")},
           "parity": parity}
    if not args.no_cpu:
        L = O.lib()
        cn = cpu_frames.shape[0]
        g = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: L.or_cksum_bench(cpu_frames.ctypes.data, 2048, cn,
                                              3, 0, g.ctypes.data, nt, reps),
            cn, args.cpu_seconds / 2)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 1496B frames x reps in 2048B slots, IPChecksum->"
                          "L4Checksum (AVX2/adc CalculateSum restated)" % cn)
    return out


def run_em1500(args, dev, torch):
    """The north star's 1500 B match point: C2's 1K-rule 5-tuple
    ExactMatch (exact_match.cc:224-244) over 1500 B packets (1496 B frames,
    SURVEY §8d) resident in 2 KB slots, the snbuf data area's size. The
    classifier reads each frame's field window only (66 B/pkt, as C2)."""
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    from oracle import oracle as O
    n = args.em1500_pkts
    # the frames' first 64 bytes (Ethernet / IPv4 with ip.length 1482 /
    # UDP or TCP), then the slab: zero payload past them
    keys, gates, hdr = P.em_workload(args.rules, n, seed=0x5EED, stride=64,
                                     frame_len=1496, pkt_seed=0x1500)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    t.sync(dev.index)
    dg = torch.empty(n, dtype=torch.int16, device=dev)
    h = torch.from_numpy(hdr).to(dev)

    def make():
        sl = torch.zeros(n * 2048, dtype=torch.uint8, device=dev)
        sl.view(n, 2048)[:, :64] = h
        return sl
    d, placement = placed_slab(
        make, lambda sl: probe_ms(lambda: t.classify(sl, 2048, n, 8192, dg), torch), torch)
    del h
    ns = 1 << 20
    sample = np.ascontiguousarray(hdr[:ns])
    del hdr
    t.classify(d, 2048, n, 8192, dg)
    torch.cuda.synchronize()
    em = oracle_em_bulk(keys, gates)
    L = O.lib()
    want = np.zeros(ns, np.uint16)
    L.or_em_process(em, sample.ctypes.data, 64, ns, 8192, want.ctypes.data)
    parity = bool((dg[:ns].cpu().numpy().view(np.uint16) == want).all())
    ms = _time_steps(lambda: t.classify(d, 2048, n, 8192, dg), args, torch, reps=leg_steps(args),
                     settle_with_step=True)
    out = {"workload": "1500B pkts (1496B frames, 2048B slots), %d-rule 5-tuple "
                       "ExactMatch, %d resident pkts" % (args.rules, n),
           "pkts": n, "ms_per_step": round(ms, 4),
           "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "kernel": "em_classify_kernel (one 32 B field window per 2 KB slot)",
           "roofline": _roof(EM_BYTES_PER_PKT, n, ms, "em1500"),
           # a 32 B window per 2 KB slot is one 64 B HBM request: the
           # shape's own rate (hbm_probe s2k32) bounds this leg
           "measured_ceiling": shape_ceiling("s2k32", n, ms),
           "placement": placement,
           "parity": "bit-exact vs oracle on %d pkts" % ns if parity else "MISMATCH"}
    if not args.no_cpu:
        cn = 1 << 18
        snb = np.zeros((cn, 2624), np.uint8)
        snb[:, 512:512 + 64] = sample[:cn]
        base = snb.ctypes.data + 512
        g = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: L.or_em_bench(em, base, 2624, cn, 8192, g.ctypes.data,
                                           nt, reps), cn, args.cpu_seconds / 2)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 1500B pkts x reps, 1K-rule 5-tuple ExactMatch, snbuf "
                          "layout (2624 B stride), 32-pkt batches" % cn)
    L.or_em_free(em)
    del d, dg
    torch.cuda.empty_cache()
    return out


def run_e2e_host(r, args, torch):
    """End-to-end rate from host memory (the reference's path starts and
    ends in mbufs): frames in snbuf-like host buffers (2624 B stride, frame
    at +512), key windows gathered into pinned memory, H2D, em_classify,
    D2H of the gates, per batch of B packets (bg_em_process_host)."""
    import ctypes as C
    from bess_amd import packets as P
    t = r["t"]
    n = 1 << 20
    _, _, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=99)
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 64] = frames
    base = snb.ctypes.data + 512
    heads = (C.c_void_p * n)(*range(base, base + n * 2624, 2624))
    out = np.zeros(n, np.uint16)
    from bess_amd._lib import lib
    res = {}
    for B in (32, 65536, n):
        lib().bg_em_process_host(t.h, heads, B, 8192, out.ctypes.data, None)
        reps = max(1, min(200, (1 << 22) // B))
        t0 = time.perf_counter()
        done = 0
        for i in range(reps):
            off = (i * B) % n
            if off + B > n:
                off = 0
            lib().bg_em_process_host(
                t.h, C.cast(C.byref(heads, off * C.sizeof(C.c_void_p)),
                            C.POINTER(C.c_void_p)),
                B, 8192, out[off:].ctypes.data, None)
            done += B
        dt = time.perf_counter() - t0
        res[str(B)] = round(done / dt / 1e6, 1)
    return {"what": "ExactMatch from host snbufs: gather windows -> pinned "
                    "-> H2D -> kernel -> D2H, synchronous per batch",
            "Mpps_by_batch": res,
            "sync_workers": run_sync_workers(args, snb, frames)}


def run_sync_workers(args, snb, frames):
    """The drop-in synchronous path under concurrent workers: T threads each
    run bg_module_run (ProcessBatch of 32 packets per call, each thread with
    its own pinned staging and HIP stream) on ONE ExactMatch module;
    aggregate Mpps by T."""
    import threading
    from bess_amd import packets as P
    from bess_amd.modules import ExactMatch
    keys, gates, _ = P.em_workload(1000, 16, seed=0x5EED)
    m = ExactMatch(fields=[{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE])
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        m.add(fields=[{"value_bin": kb[a:c]} for a, c in cut], gate=int(g))
    n_per = 1 << 14
    base = snb.ctypes.data + 512
    heads = base + 2624 * np.arange(len(frames), dtype=np.uintp)
    m.run(heads[:n_per], burst=32)  # warm: staging, streams, table sync
    out = {}
    for T in (1, 2, 4, 8, 16):
        rots = [np.ascontiguousarray(np.roll(heads, -i * 7919)[:n_per]) for i in range(T)]
        for r_ in rots:
            m.run(r_[:256], burst=32)
        ths = [threading.Thread(target=m.run, args=(rots[i],), kwargs={"burst": 32})
               for i in range(T)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        out[str(T)] = round(T * n_per / dt / 1e6, 2)
    return {"what": "T worker threads, bg_module_run (32-packet ProcessBatch, "
                    "synchronous) on one ExactMatch module, 1000 rules",
            "Mpps_by_threads": out,
            "x4_over_1": round(out["4"] / out["1"], 2)}


def _pipe_rate(make_pipe, heads, lens, threads, reps, burst=32):
    """aggregate Mpps of `threads` BESS-style workers, each with its own
    bg_pipe over the shared packet pool (its own rotation of it), each
    running the native worker loop (bg_pipe_run) `reps` times"""
    import threading
    n = len(heads)
    pipes = [make_pipe() for _ in range(threads)]
    rots = [np.roll(heads, -(i * n) // threads) for i in range(threads)]
    lrots = [None if lens is None else np.roll(lens, -(i * n) // threads)
             for i in range(threads)]
    for p, h, ln in zip(pipes, rots, lrots):  # warm: staging, tables, caches
        p.run(h[:65536], None if ln is None else ln[:65536])
    errs = []

    def work(p, h, ln):
        try:
            for _ in range(reps):
                p.run(h, ln, burst=burst)
        except Exception as e:  # reported below
            errs.append(e)
    ths = [threading.Thread(target=work, args=a) for a in zip(pipes, rots, lrots)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    for p in pipes:
        p.close()
    if errs:
        raise errs[0]
    return round(threads * reps * n / dt / 1e6, 1)


def run_e2e_pipe(args, torch):
    """End-to-end from host memory through the aggregation queue (bg_pipe):
    packets in snbuf-like host buffers (2624 B objects, frame at +512) are
    submitted 32 per ProcessBatch call by native worker loops; each worker's
    pipe gathers the bytes the device reads into pinned slots of `batch`
    packets and runs H2D -> kernel -> D2H on 4 streams; gates come back in
    submission order. Parity: the gates of one pass vs the oracle."""
    from bess_amd import packets as P
    from bess_amd.modules import ExactMatch, L4Checksum, Pipe
    from oracle import oracle as O
    out = {"burst": 32, "depth": 4,
           "host_cpus_used": "1 worker thread per pipe"}
    # ExactMatch, C2 rules, 64 B packets
    n = 1 << 20
    keys, gates, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=77)
    fields = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]
    m = ExactMatch(fields=fields)
    om = O.OracleExactMatch(fields=fields)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        v = [{"value_bin": kb[a:c]} for a, c in cut]
        m.add(fields=v, gate=int(g))
        om.add(fields=v, gate=int(g))
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 64] = frames
    heads = snb.ctypes.data + 512 + 2624 * np.arange(n, dtype=np.uintp)
    want = om.process(frames, 64, n)
    del frames
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    em = {}
    # ring: slots go to the module's persistent kernel (the plugin's shape,
    # 8 x 1024 in flight per worker); launch: H2D/kernel/D2H per slot
    for mode, batch, depth in (("ring", 1024, 8), ("launch", 4096, 4),
                               ("launch", 65536, 4)):
        key = "%s_batch%d_depth%d" % (mode, batch, depth)
        with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
            p = Pipe(m, batch=batch, depth=depth)
            em["parity_" + key] = bool((p.run(heads) == want).all())
            p.close()
            rates = {}
            for th in [int(x) for x in args.pipe_threads.split(",")]:
                rates[str(th)] = _pipe_rate(
                    lambda: Pipe(m, batch=batch, depth=depth), heads, None, th,
                    reps=2 if th == 1 else 4)
        em["Mpps_by_threads_" + key] = rates
        # the staged 16 B field window in, the 2 B gate out
        em["pcie_16_threads_" + key] = pcie(rates.get("16"), 16, 2)
    out["ExactMatch_64B"] = em
    del snb
    # WildcardMatch, C4 rules (100 K over 8 masks), IMIX frames: the heavier
    # classifier, where the device's per-packet work outweighs the gather
    # (compare the C4 entry's cpu_baseline on the same cores)
    from bess_amd.modules import WildcardMatch
    n = 1 << 18
    rk, rm, prio, wg, wf, _ = P.wm_workload(100000, n, stride=2048)
    mw = WildcardMatch(fields=fields)
    ow = O.OracleWildcardMatch(fields=fields)
    for k, mk, pr, g in zip(rk, rm, prio, wg):
        kb, mb = k.tobytes(), mk.tobytes()
        kw = dict(gate=int(g), priority=int(pr),
                  values=[{"value_bin": kb[a:c]} for a, c in cut],
                  masks=[{"value_bin": mb[a:c]} for a, c in cut])
        mw.add(**kw)
        ow.add(**kw)
    want = ow.process(wf, 2048, n)
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 2048] = wf
    del wf
    heads = snb.ctypes.data + 512 + 2624 * np.arange(n, dtype=np.uintp)
    p = Pipe(mw, batch=65536, depth=4)
    wmr = {"parity": bool((p.run(heads) == want).all())}
    p.close()
    rates = {}
    for th in [int(x) for x in args.pipe_threads.split(",")]:
        rates[str(th)] = _pipe_rate(lambda: Pipe(mw, batch=65536, depth=4), heads,
                                    None, th, reps=4)
    wmr["Mpps_by_threads_batch65536"] = rates
    wmr["pcie_16_threads"] = pcie(rates.get("16"), 16, 2)
    out["WildcardMatch_IMIX_100K"] = wmr
    del snb
    # L4Checksum (recompute), 1500 B packets: frames H2D, header lines back
    n = 1 << 17
    cf = P.cksum_workload(n, frame_len=1496)
    ref = cf.copy()
    _, l4w = O.cksum_process(ref, 2048, n, 2, False)
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 2048] = cf
    heads = snb.ctypes.data + 512 + 2624 * np.arange(n, dtype=np.uintp)
    lens = np.full(n, 1496, np.uint16)
    mk = L4Checksum(verify=False)
    p = Pipe(mk, batch=8192, depth=4, span=1504)
    g = p.run(heads, lens)
    p.close()
    ck = {"parity": bool((g == l4w).all() and
                         (snb[:, 512:512 + 1496] == ref[:, :1496]).all())}
    rates = {}
    for th in [int(x) for x in args.pipe_threads.split(",")]:
        rates[str(th)] = _pipe_rate(
            lambda: Pipe(mk, batch=8192, depth=4, span=1504), heads, lens, th,
            reps=4)
    ck["Mpps_by_threads_batch8192"] = rates
    ck["pcie_16_threads"] = pcie(rates.get("16"), 1504, 130)
    out["L4Checksum_1500B"] = ck
    return out


def run_plugin_pipeline(args):
    """The bessd drop-in as a BESS user gets it: the ExactMatch plugin
    (integration/bessd/exact_match_gpu.cc, deferred datapath: ProcessBatch
    enqueues into its worker's pipe, the module's task emits, as Queue does)
    compiled against the header shell, driven by the shell's worker loop
    (tests/bessd_shell/drive.cc `pipeline`): Source -> ExactMatch -> Sink,
    32-packet batches, T pinned workers, each over its own slice of the
    pool, EmitPacket to connected gates. The same pool and slicing as the
    C2 cpu_baseline (2^18 64 B packets in 2624 B snbuf objects, 1000
    rules), so the two rates compare on the same cores."""
    import subprocess
    import tempfile
    from bess_amd import packets as P
    from bess_amd import pb
    from oracle import oracle as O
    drive = args.drive or os.path.join(ROOT, "tests", "bessd_shell", "build", "drive")
    if not os.path.exists(drive):
        return "skipped: %s not built" % drive
    n = 1 << 18
    keys, gates, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=77)
    fields = [{"offset": o, "num_bytes": sz} for o, sz in P.FIVE_TUPLE]
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    om = O.OracleExactMatch(fields=fields)
    script = ["create ExactMatch " +
              pb.dict_to_protobuf(pb.ExactMatchArg, {"fields": fields})
              .SerializeToString().hex()]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        v = [{"value_bin": kb[a:c]} for a, c in cut]
        om.add(fields=v, gate=int(g))
        script.append("cmd add " + pb.dict_to_protobuf(
            pb.ExactMatchCommandAddArg, {"gate": int(g), "fields": v})
            .SerializeToString().hex())
    want = om.process(frames, 64, n)
    script += ["connect %d" % g for g in range(65)]
    threads = [int(x) for x in args.pipe_threads.split(",")]
    res, parity, pipe_stats, cpu_res, cpu_parity = {}, {}, {}, {}, {}
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "frames.bin")
        frames.tofile(path)
        kpath, gpath = os.path.join(td, "keys.bin"), os.path.join(td, "gates.bin")
        np.ascontiguousarray(keys, dtype=np.uint8).tofile(kpath)
        np.ascontiguousarray(gates, dtype=np.uint16).tofile(gpath)
        script.append("frames %s 64 %d" % (path, n))
        script.append("cpu_em %s %s %d %d" % (kpath, gpath, len(keys), keys.shape[1]))
        for t in threads:
            reps = 64 if t == 1 else 256
            sc = script + ["pipeline %d 2 0 0 0" % t,  # warm: lanes, tables
                           "pipeline %d %d 0 0 0" % (t, reps),
                           # the CPU baseline in the same harness: the
                           # restated reference ProcessBatch on the workers
                           "pipeline_cpu %d 2" % t, "pipeline_cpu %d %d" % (t, reps)]
            r = subprocess.run([drive, "run"], input="\n".join(sc) + "\n",
                               capture_output=True, text=True, timeout=600)
            lines = r.stdout.splitlines()
            stats = [x for x in lines if x.startswith("pipeline")]
            outs = [x for x in lines if x.startswith("out")]
            if r.returncode or len(stats) < 4 or len(outs) < 4:
                res[str(t)] = "failed: rc %d %s" % (r.returncode, r.stderr[-300:])
                continue
            res[str(t)] = round(float(stats[1].split()[1]), 1)
            cpu_res[str(t)] = round(float(stats[3].split()[1]), 1)
            pst = [x for x in lines if x.startswith("stats")]
            cyc = [x for x in lines if x.startswith("cycles")]
            if pst:
                pipe_stats[str(t)] = pst[-1][6:]
            if len(cyc) >= 4:
                pipe_stats[str(t) + "_cycles_gpu"] = cyc[1][7:]
                pipe_stats[str(t) + "_cycles_cpu"] = cyc[3][7:]
            # EmitPacket to DROP_GATE (the default gate) drops: "D"
            exp = ["D" if int(w) >= 8192 else str(int(w)) for w in want]
            parity[str(t)] = outs[1].split()[1:] == exp
            cpu_parity[str(t)] = outs[3].split()[1:] == exp
    # worker 0's pipe counters and cycles: diagnostics, to stderr with
    # --diag only (the driver's record keeps ~8 KB of stdout + stderr: the
    # line's last sections must fit)
    if args.diag:
        log("e2e_plugin worker0_pipe_stats " + json.dumps(pipe_stats))
    return {"what": "Source -> ExactMatch plugin (deferred: per-worker bg_pipe, "
                    "task emits) -> Sink, 32-pkt batches, 1000 rules, %d 64B "
                    "pkts in 2624 B snbufs split over the workers as the "
                    "cpu_baseline splits them" % n,
            "Mpps_by_workers": res,
            "pipe": {"mode": "ring (bg_em_ring, one lane per worker)",
                     "batch": 1024, "depth": 8},
            "parity": parity,
            "pcie_16_workers": pcie(res.get("16"), 16, 2),
            "cpu_same_harness": {
                "what": "the same Source -> Sink workers with the restated "
                        "reference ExactMatch::ProcessBatch (oracle: head_data() "
                        "per packet, MakeKeys, CuckooMap/CRC32C Find, EmitPacket) "
                        "in place of the plugin",
                "Mpps_by_workers": cpu_res, "parity": cpu_parity}}


def run_plugin_pool(args):
    """bessd plugins on a bounded packet pool (tests/bessd_shell `pool`):
    16 workers' Sources allocate every 32-packet batch from 262,144 snbufs
    (bessd's --buffers default, core/opts.cc:127) and copy the frame in, as
    Source copies its template; Sinks free the packets back. WildcardMatch
    (C4-style rules, IMIX frames in 2 KB slots) and L4Checksum (1496 B frames)
    plugins on the deferred datapath, each worker's pipe held to its share
    of the pool (GpuModule::PipeBudget). Mpps over the packets the Sinks
    took over the timed passes (the Sources copy each frame's length, from
    its IPv4 header); parity of the last pass against the oracle."""
    import subprocess
    import tempfile
    from bess_amd import packets as P
    from bess_amd import pb
    from oracle import oracle as O
    drive = args.drive or os.path.join(ROOT, "tests", "bessd_shell", "build", "drive")
    if not os.path.exists(drive):
        return "skipped: %s not built" % drive
    n = 1 << 17
    fields = [{"offset": o, "num_bytes": sz} for o, sz in P.FIVE_TUPLE]
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    out = {"pool": 262144, "workers": 16, "pkts_per_pass": n}
    with tempfile.TemporaryDirectory() as td:
        for name in ("WildcardMatch", "L4Checksum"):
            if name == "WildcardMatch":
                nr = 100000
                rk, rm, prio, wg, frames, _ = P.wm_workload(nr, n, stride=2048)
                ow = O.OracleWildcardMatch(fields=fields)
                script = ["create WildcardMatch " + pb.dict_to_protobuf(
                    pb.WildcardMatchArg, {"fields": fields}).SerializeToString().hex()]
                for k, mk, p, g in zip(rk, rm, prio, wg):
                    kb, mb = k.tobytes(), mk.tobytes()
                    a = dict(gate=int(g), priority=int(p),
                             values=[{"value_bin": kb[x:y]} for x, y in cut],
                             masks=[{"value_bin": mb[x:y]} for x, y in cut])
                    ow.add(**a)
                    script.append("cmd add " + pb.dict_to_protobuf(
                        pb.WildcardMatchCommandAddArg, a).SerializeToString().hex())
                script += ["connect %d" % g for g in range(64)]
                want = ow.process(frames, 2048, n)
                exp = [str(int(w)) if int(w) < 64 else "D" for w in want]
                # the CPU baseline in the same harness: the restated
                # reference WildcardMatch::ProcessBatch on the same workers
                wpaths = [os.path.join(td, x) for x in ("k", "m", "p", "g")]
                for arr, pth, dt in zip((rk, rm, prio, wg), wpaths,
                                        (np.uint8, np.uint8, np.int32, np.uint16)):
                    np.ascontiguousarray(arr, dtype=dt).tofile(pth)
                script.append("cpu_wm %s %s %s %s %d" % (*wpaths, nr))
            else:
                # UDP only: the reference's L4Checksum never emits (nor
                # frees) a TCP packet in calculate mode (P8), so a TCP share
                # would drain the pool pass by pass (tests/test_bessd_wrappers
                # counts that leak with mixed frames)
                frames = P.cksum_workload(n, frame_len=1496, udp_frac=1.0)
                ref = frames.copy()
                _, l4w = O.cksum_process(ref, 2048, n, 2, False)
                script = ["create L4Checksum -", "connect 0", "connect 1"]
                exp = ["-" if int(w) == 0xFFFF else str(int(w)) for w in l4w]
                # the CPU baseline in the same harness: the restated
                # reference L4Checksum::ProcessBatch (AVX2/adc CalculateSum)
                script.append("cpu_l4 0")
            path = os.path.join(td, "f.bin")
            frames.tofile(path)
            # enough passes for the steady state (the first pass opens the
            # workers' pipes; a pass of 2^17 packets is ~10 ms)
            reps = 40 if name == "WildcardMatch" else 20
            script += ["frames %s 2048 %d" % (path, n), "pool 262144",
                       "pipeline 16 1 0 0 0", "sleep 3000",  # (the run-time compile)
                       "pipeline 16 %d 0 0 0" % reps]
            script += ["pipeline_cpu 16 1", "pipeline_cpu 16 %d" % reps]
            r = subprocess.run([drive, "run"], input="\n".join(script) + "\n",
                               capture_output=True, text=True, timeout=600)
            lines = r.stdout.splitlines()
            stats = [x for x in lines if x.startswith("pipeline")]
            outs = [x for x in lines if x.startswith("out")]
            pools = [x.split() for x in lines if x.startswith("pool")]
            if r.returncode or len(stats) < 2 or len(outs) < 2:
                out[name] = "failed: rc %d %s" % (r.returncode, r.stderr[-300:])
                continue
            out[name] = {"Mpps": round(float(stats[1].split()[1]), 1),
                         "parity": outs[1].split()[1:] == exp,
                         "pool_after": "%s of %s back" % (pools[-1][1], pools[-1][2]),
                         "never_emitted_per_pass": exp.count("-"),
                         "source_waits": int(pools[-1][3])}
            # worker 0's pipe counters and TSC cycles per packet of the timed
            # passes (where the host side's time goes), the plugin's and the
            # restated reference's side by side
            st = [x for x in lines if x.startswith("stats")]
            cyc = [x for x in lines if x.startswith("cycles")]
            if args.diag and len(st) >= 2:
                log("e2e_plugin_pool %s pipe_w0 %s" % (name, st[1][6:]))
            if len(st) >= 2:  # the submit cost per packet (the copy it saves)
                f = st[1].split()
                out[name]["submit_cyc_per_pkt"] = float(f[f.index("submit_cyc_per_pkt") + 1])
                out[name]["poll_cyc_per_pkt"] = float(f[f.index("poll_cyc_per_pkt") + 1])

            def phases(line):
                f = line.split()
                return {k: float(f[f.index(k) + 1]) for k in
                        ("source", "proc", "sink", "task") if k in f}
            if len(cyc) >= 4:
                out[name]["w0_cycles_per_pkt"] = {
                    "plugin": phases(cyc[1]), "reference": phases(cyc[3]),
                    "tsc_ghz": float(cyc[1].split()[-1])}
            # the frames read in place from the registered pool (L4Checksum:
            # 1504 B of 16 B loads per 1496 B frame, the checksum word and
            # gate back) or the staged 16 B field window (WildcardMatch)
            out[name]["pcie"] = pcie(out[name]["Mpps"], *((16, 2) if name == "WildcardMatch"
                                                          else (1504, 4)))
            if name == "WildcardMatch":
                out[name]["rules"] = nr
            if len(stats) >= 4 and len(outs) >= 4:
                out[name]["cpu_same_harness"] = {
                    "what": "the same pool, Sources and Sinks with the restated "
                            "reference %s::ProcessBatch in place of the plugin" % name,
                    "Mpps": round(float(stats[3].split()[1]), 1),
                    "parity": outs[3].split()[1:] == exp}
    return out


def clock_settle(args, torch, fn=None):
    """Untimed, before a leg's warm-up: ~args.settle_ms of back-to-back
    device work. A leg starts after host work (its table build, the parity
    check) that left the GPU idle, and the first ~25 launches over a fresh
    slab then run up to 14 % slow (profiles/r05/ck_timing_r05i.json): with
    the driver's --warmup 5 the timed region would measure that ramp, not
    the kernel. `fn`: the leg's own launch, for legs whose launches leave
    their input as it was (classifiers -- the headline among them, since
    round 6 -- and idempotent checksums); otherwise an in-place multiply
    over 1 GB (legs that modify packets in place keep their launch budget).
    The work must stream HBM: after ~100 ms of it, launches 5-25 of C2's
    kernel ran 0.1667-0.1684 ms against 0.1652-0.1654 after its own
    launches, 0.1723-0.1738 after the same multiply over 64 MB (which stays
    in the Infinity Cache; the round-5 settle) and 0.185-0.193 after none
    (profiles/r06/first_launch_settle_r06ad.json)."""
    if args.settle_ms <= 0:
        return
    x = None
    if fn is None:
        x = torch.ones(256 << 20, dtype=torch.float32, device="cuda")
        fn = lambda: x.mul_(1.0)  # noqa: E731
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.settle_ms:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    del x


def leg_steps(args):
    """timed launches of a configuration leg other than the headline: at
    least 100 (the driver's --steps 20 timed C4's 2 KB-slot leg 10-17 %
    slower than 200 steps did: profiles/r05/bench_line_driver_args_before_
    floor.json against bench_line_driver_args.json); the headline times
    exactly --steps"""
    return max(args.steps, 100)


def _time_steps(step, args, torch, settle_with_step=False, reps=10):
    """warmup, then ms per launch over `reps` launches (HIP events on the
    launching stream); settle_with_step: the step leaves its input as it
    was, so clock_settle runs it"""
    clock_settle(args, torch, step if settle_with_step else None)
    for _ in range(max(3, args.warmup // 4)):
        step()
    torch.cuda.synchronize()
    timer = Timer(torch)
    timer.start()
    for _ in range(reps):
        step()
    return timer.stop_ms() / reps


def _roof(bytes_per_pkt, n, ms, key=None):
    gbs = bytes_per_pkt * n / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
         "bytes_per_pkt": bytes_per_pkt}
    if key:
        r["traffic"] = traffic_gbs(key, ms)
        r["traffic_bytes_per_launch"] = load_traffic(key)
    return r


def _snbuf_sample(frames, n):
    """the first n frames copied into snbuf-like objects (2624 B, +512):
    the CPU reference's memory layout"""
    w = min(frames.shape[1], 2048)
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + w] = frames[:n, :w]
    return snb


def run_hashlb(args, dev, torch):
    """HashLB (core/modules/hash_lb.cc) on the C2 slab: 16M 64 B packets,
    8 gates; l4 mode (the default) and a 5-tuple fields mode"""
    from bess_amd import packets as P
    from bess_amd.modules import HashLB
    from oracle import oracle_more as OM
    n = args.pkts
    _, _, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=5)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    g = torch.empty(n, dtype=torch.int16, device=dev)
    out = {"workload": "HashLB: 64B pkts (64B slots), 8 gates, %d resident "
                       "pkts" % n, "pkts": n}
    five = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]
    for name, kw in (("l4", dict(mode="l4")), ("fields_5tuple", dict(fields=five))):
        m = HashLB(gates=list(range(8)), **kw)
        o = OM.OracleHashLB(gates=list(range(8)), **kw)
        m.process_device(d, 64, n, g)
        torch.cuda.synchronize()
        k = min(n, 1 << 20)
        parity = bool((g[:k].cpu().numpy().view(np.uint16) ==
                       o.process(frames, 64, k)).all())
        ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch,
                         settle_with_step=True)
        out[name] = {"ms_per_step": round(ms, 4),
                     "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
                     "roofline": _roof(EM_BYTES_PER_PKT, n, ms,
                                       "hashlb" if name == "l4" else None),
                     "parity": "bit-exact vs oracle on %d pkts" % k
                               if parity else "MISMATCH"}
        if not args.no_cpu:
            cn = 1 << 18
            snb = _snbuf_sample(frames, cn)
            og = np.zeros(cn, np.uint16)
            gt = np.array(o.gates_, np.uint16)
            L = OM.mlib()
            threads, res = cpu_rate(
                lambda nt, reps: L.or_hashlb_bench(
                    o.mode, o._em, o.hash_len, gt.ctypes.data, 8, snb.ctypes.data + 512,
                    2624, cn, og.ctypes.data, nt, reps), cn, args.cpu_seconds / 3)
            out[name]["cpu_baseline"] = cpu_baseline(
                res, threads, "%d 64B pkts x reps in snbuf layout, HashLB %s "
                              "(SSE4.2 CRC32C)" % (cn, name))
    return out


def run_acl(args, dev, torch):
    """ACL (core/modules/acl.cc) on the C2 slab: 16M 64 B packets, random
    ordered rule lists (prefixes /0../32, port wildcards, 30 % drop rules),
    70 % of packets derived from some rule's tuple"""
    import sys as _s
    _s.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_acl import workload
    from bess_amd.modules import ACL
    from oracle import oracle_more as OM
    n = args.pkts
    out = {"workload": "ACL: 64B pkts (64B slots), %d resident pkts, first-"
                       "match over an ordered rule list" % n, "pkts": n}
    g = torch.empty(n, dtype=torch.int16, device=dev)
    for nr in (100, 1000):
        rules, frames = workload(nr, n, seed=nr)
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        m = ACL(rules=rules)
        o = OM.OracleACL(rules=rules)
        m.process_device(d, 64, n, g)
        torch.cuda.synchronize()
        k = min(n, 1 << 18)
        parity = bool((g[:k].cpu().numpy().view(np.uint16) ==
                       o.process(frames, 64, k)).all())
        ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch,
                         settle_with_step=True)
        e = {"ms_per_step": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
             "roofline": _roof(EM_BYTES_PER_PKT, n, ms, "acl"),
             "parity": "bit-exact vs oracle on %d pkts" % k if parity else "MISMATCH"}
        if not args.no_cpu:
            cn = 1 << 16
            snb = _snbuf_sample(frames, cn)
            threads, res = cpu_rate(
                lambda nt, reps: o.bench(snb.ctypes.data + 512, 2624, cn, nt, reps),
                cn, args.cpu_seconds / 4)
            e["cpu_baseline"] = cpu_baseline(
                res, threads, "%d 64B pkts x reps in snbuf layout, %d-rule ACL"
                              % (cn, nr))
        out["rules_%d" % nr] = e
        del d
    return out


def run_iplookup(args, dev, torch):
    """IPLookup (core/modules/ip_lookup.cc) on the C2 slab: 16M 64 B packets,
    10K routes (/8../24, 5 % /25../32, nested), half the destinations inside
    a route; the default DIR-16-8-8 tables (tbl16 staged in LDS, tbl2 groups
    in L2; DIR-24-8 only past 32 K groups)"""
    import sys as _s
    _s.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_iplookup import build, dsts_inside, frames_to, routes
    from oracle import oracle as O
    n = args.pkts
    rng = np.random.default_rng(0x5EED)
    rt = routes(10000, rng, 0.05)
    m, o = build(rt, max_rules=20000, max_tbl8s=4096)
    dst = np.concatenate([dsts_inside(rt, n // 2, rng),
                          rng.integers(0, 1 << 32, n - n // 2, dtype=np.uint64)])
    rng.shuffle(dst)
    frames = frames_to(dst)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    g = torch.empty(n, dtype=torch.int16, device=dev)
    m.process_device(d, 64, n, g)
    torch.cuda.synchronize()
    k = min(n, 1 << 20)
    parity = bool((g[:k].cpu().numpy().view(np.uint16) ==
                   o.process(frames, 64, k)).all())
    ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch,
                         settle_with_step=True)
    out = {"workload": "IPLookup: 64B pkts (64B slots), %d resident pkts, 10K "
                       "routes, DIR-16-8-8 (tbl16 in LDS)" % n, "pkts": n,
           "routes": len(o.rules),
           "ms_per_step": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "roofline": _roof(EM_BYTES_PER_PKT, n, ms, "iplookup"),
           "parity": "bit-exact vs oracle on %d pkts" % k if parity else "MISMATCH"}
    if not args.no_cpu:
        from oracle import oracle_more as OM
        cn = 1 << 18
        snb = _snbuf_sample(frames, cn)
        tab = o.dir24()
        og = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: OM.mlib().or_dir24_bench(
                tab, snb.ctypes.data + 512, 2624, cn, o.default_gate,
                og.ctypes.data, nt, reps), cn, args.cpu_seconds / 3)
        OM.mlib().or_dir24_free(tab)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 64B pkts x reps in snbuf layout, 10K routes, "
                          "rte_lpm's DIR-24-8 lookup restated (DPDK absent)" % cn)
    return out


def run_update_ttl(args, dev, torch):
    """UpdateTTL (core/modules/update_ttl.cc) in place on the C2 slab: 16M
    64 B packets, TTL 200 (every timed launch decrements and rewrites: the
    launches stay below 200). Bytes/pkt: 64 B header line read + the same
    line written back whole (a partial-line write costs HBM a read-modify-
    write, measured slower) + 2 B gate = 130."""
    from bess_amd import packets as P
    from bess_amd.modules import UpdateTTL
    from oracle import oracle_more as OM
    n = args.pkts
    _, _, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=11)
    frames[:, 22] = 200
    k = min(n, 1 << 20)
    ref = frames[:k].copy()
    want = OM.update_ttl_process(ref, 64, k)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    g = torch.empty(n, dtype=torch.int16, device=dev)
    m = UpdateTTL()
    m.process_device(d, 64, n, g)
    torch.cuda.synchronize()
    parity = bool((g[:k].cpu().numpy().view(np.uint16) == want).all() and
                  (d[:k * 64].cpu().numpy().reshape(k, 64) == ref).all())
    reps = 10
    warm = max(3, args.warmup // 4)
    assert reps + warm + 1 < 199
    ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
    out = {"workload": "UpdateTTL: 64B pkts (64B slots), %d resident pkts, in "
                       "place" % n, "pkts": n, "ms_per_step": round(ms, 4),
           "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "roofline": _roof(130, n, ms, "ttl"),
           "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                     if parity else "MISMATCH"}
    if not args.no_cpu:
        cn = 1 << 18
        snb = _snbuf_sample(ref, cn)
        snb[:, 512 + 22] = 255  # every rep decrements (<= 250 reps)
        og = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: OM.mlib().or_update_ttl_bench(
                snb.ctypes.data + 512, 2624, cn, og.ctypes.data, nt, reps),
            cn, args.cpu_seconds / 3, max_reps=120)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 64B pkts x reps in snbuf layout, in place" % cn)
    return out


def run_rewrite(args, dev, torch):
    """Rewrite (core/modules/rewrite.cc) over 16M packet slots: 4 templates
    of 60 B (the Source -> Rewrite front of a BESS pipeline), round robin;
    slots of 192 B (128 B headroom + data). Bytes/pkt: the 64 B the
    reference's 32-byte-block copy writes + data_off (2 B) + length (4 B) =
    70, all writes."""
    from bess_amd import packets as P
    from bess_amd.modules import Rewrite
    from oracle import oracle_more as OM
    n, stride = args.pkts, 192
    _, _, fr = P.em_workload(4, 4, seed=0x5EED, pkt_seed=3)
    ts = [fr[i, :60].tobytes() for i in range(4)]
    m, o = Rewrite(templates=ts), OM.OracleRewrite(ts)
    d = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    dh = torch.zeros(n, dtype=torch.int16, device=dev)
    dl = torch.zeros(n, dtype=torch.int32, device=dev)
    k = min(n, 1 << 18)
    m.process_device(d, stride, n, dh, dl)  # all n (PMC passes average every launch)
    torch.cuda.synchronize()
    m.clear()
    m.add(templates=ts)  # the turn back at 0 for the timed calls
    ref = np.zeros((k, stride), np.uint8)
    oh, ol = np.zeros(k, np.uint16), np.zeros(k, np.uint32)
    o.process(ref, stride, k, oh, ol)
    parity = bool((d[:k * stride].cpu().numpy().reshape(k, stride) == ref).all() and
                  (dh[:k].cpu().numpy().view(np.uint16) == oh).all() and
                  (dl[:k].cpu().numpy().view(np.uint32) == ol).all())
    # Rewrite reads no packet bytes, so its own launch settles the clocks and
    # any number of launches times the same work
    ms = _time_steps(lambda: m.process_device(d, stride, n, dh, dl), args, torch,
                     reps=leg_steps(args), settle_with_step=True)
    out = {"workload": "Rewrite: 4 templates of 60B round robin into %d resident "
                       "192B packet slots" % n, "pkts": n, "ms_per_step": round(ms, 4),
           "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "roofline": _roof(70, n, ms, "rewrite"),
           "parity": "bit-exact (slots, data_off, lengths) vs oracle on %d pkts" % k
                     if parity else "MISMATCH"}
    if not args.no_cpu:
        cn = 1 << 18
        snb = np.zeros((cn, 2624), np.uint8)
        hh, ll = np.zeros(cn, np.uint16), np.zeros(cn, np.uint32)
        busy, done, i = 0.0, 0, 0
        while busy < args.cpu_seconds / 3 or i < 2:
            t0 = time.perf_counter()
            OM.mlib().or_rewrite_process(o.h, snb.ctypes.data, 2624, cn, 128,
                                         hh.ctypes.data, ll.ctypes.data)
            busy += time.perf_counter() - t0
            done += cn
            i += 1
        out["cpu_baseline"] = cpu_baseline({1: done / busy / 1e6}, 1,
                                           "%d packets x %d passes in snbuf layout, "
                                           "1 thread" % (cn, i))
    return out


def nat_pairs():
    """16 pairs: 8 /16s 10.i.0.0 -> 100.i.0.0 then their images mapped
    back, so every launch translates the same packets again (steady state)"""
    pairs = []
    for back in (0, 1):
        for i in range(8):
            a, b = "10.%d" % i, "100.%d" % i
            if back:
                a, b = b, a
            pairs.append({"int_range": {"start": a + ".0.0", "end": a + ".255.255"},
                          "ext_range": {"start": b + ".0.0", "end": b + ".255.255"}})
    return pairs


def run_static_nat(args, dev, torch):
    """StaticNAT (core/modules/static_nat.cc) forward direction in place on
    the C2 slab: 16M 64 B packets, 16 address pairs, half the sources inside
    a pair (translated, IP + L4 checksums updated), half outside (all 16
    pairs scanned). Bytes/pkt: 64 B line read + 2 B gate + the 64 B line
    written back for the packets the op changes (the kernel writes back only
    those: 66 + 64 x the translated fraction, measured on the parity sample;
    every packet written back, as before round 6, was 130)."""
    from bess_amd import packets as P
    from bess_amd.modules import StaticNAT
    from oracle import oracle_more as OM
    n = args.pkts
    _, _, frames = P.em_workload(args.rules, n, seed=0x5EED, pkt_seed=13)
    rng = np.random.default_rng(13)
    hit = rng.random(n) < 0.5
    frames[hit, 26] = 10
    frames[hit, 27] = rng.integers(0, 8, int(hit.sum()), dtype=np.uint8)
    k = min(n, 1 << 20)
    ref = frames[:k].copy()
    want = OM.OracleStaticNAT(pairs=nat_pairs()).process(ref, 64, k)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    g = torch.empty(n, dtype=torch.int16, device=dev)
    m = StaticNAT(pairs=nat_pairs())
    m.process_device(d, 64, n, g)
    torch.cuda.synchronize()
    parity = bool((g[:k].cpu().numpy().view(np.uint16) == want).all() and
                  (d[:k * 64].cpu().numpy().reshape(k, 64) == ref).all())
    changed = float((ref != frames[:k]).any(1).mean())
    bpp = round(66 + 64 * changed, 2)
    ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
    out = {"workload": "StaticNAT forward: 64B pkts (64B slots), %d resident "
                       "pkts, 16 pairs, 50%% translated, in place" % n,
           "pkts": n, "ms_per_step": round(ms, 4),
           "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "roofline": _roof(bpp, n, ms, "nat"),
           "translated_fraction": round(changed, 4),
           "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                     if parity else "MISMATCH"}
    if not args.no_cpu:
        cn = 1 << 18
        snb = _snbuf_sample(frames, cn)
        o = OM.OracleStaticNAT(pairs=nat_pairs())
        threads, res = cpu_rate(
            lambda nt, reps: o.bench(snb.ctypes.data + 512, 2624, cn, nt, reps),
            cn, args.cpu_seconds / 3)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 64B pkts x reps in snbuf layout, 16 pairs, in "
                          "place (translations flip back and forth)" % cn)
    return out


def run_dnat(args, dev, torch):
    """NAT (core/modules/nat.cc), established flows -- the device-only path:
    64K internal TCP/UDP flows mapped in a setup batch (the host's port
    search), then fresh copies of a 16M-packet 64 B slab of those flows
    translated forward (one fused lookup + Stamp + timestamp refresh pass,
    then the 4-byte miss count read back). Bytes/pkt: 64 B line read + 64 B
    written + 2 B gate = 130."""
    from bess_amd import packets as P
    from bess_amd.modules import NAT
    from oracle import oracle_more as OM
    nflow, n = 1 << 16, 1 << 24
    _, _, flows = P.em_workload(16, nflow, seed=0x5EED, pkt_seed=17)
    zero = (flows[:, 34] == 0) & (flows[:, 35] == 0)
    flows[zero, 35] = 1                        # port 0 never maps
    rng = np.random.default_rng(17)
    slab = flows[rng.integers(0, nflow, n)]
    ext = [{"ext_addr": "100.64.0.1"}, {"ext_addr": "100.64.0.2"}]
    m, o = NAT(ext_addrs=ext, seed=0x5EED), OM.OracleNAT(ext_addrs=ext, seed=0x5EED)
    t0 = 10 ** 12
    d_setup = torch.from_numpy(flows.reshape(-1).copy()).to(dev)
    g = torch.empty(n, dtype=torch.int16, device=dev)
    m.process_device(d_setup, 64, nflow, g, t0)
    o.process(flows.copy(), 64, nflow, 0, t0)
    reps = 10
    src = torch.from_numpy(slab.reshape(-1)).to(dev)
    copies = [src.clone() for _ in range(reps + 1)]
    torch.cuda.synchronize()
    k = 1 << 18
    ref = slab[:k].copy()
    want = o.process(ref, 64, k, 0, t0 + 1)
    m.process_device(copies[0], 64, n, g, t0 + 1)
    torch.cuda.synchronize()
    parity = bool((g[:k].cpu().numpy().view(np.uint16) == want).all() and
                  (copies[0][:k * 64].cpu().numpy().reshape(k, 64) == ref).all())
    clock_settle(args, torch)
    timer = Timer(torch)
    timer.start()
    for i in range(reps):
        m.process_device(copies[i + 1], 64, n, g, t0 + 2 + i)
    ms = timer.stop_ms() / reps
    cpu = None
    if not args.no_cpu:
        # one worker (the reference NAT map is not shared between workers):
        # fresh copies of the sample per pass, copies untimed
        cn = 1 << 18
        snb0 = _snbuf_sample(slab, cn)
        snb = snb0.copy()
        og = np.zeros(cn, np.uint16)
        busy, done, i = 0.0, 0, 0
        while busy < args.cpu_seconds / 3 or i < 2:
            snb[:] = snb0
            t0c = time.perf_counter()
            OM.mlib().or_nat_process(o.h, snb.ctypes.data + 512, 2624, cn, 0,
                                     t0 + 100 + i, og.ctypes.data)
            busy += time.perf_counter() - t0c
            done += cn
            i += 1
        rate = done / busy / 1e6
        cpu = cpu_baseline({1: rate}, 1, "%d 64B pkts x %d passes in snbuf "
                           "layout, established flows, 1 worker (one NAT map)"
                           % (cn, i))
    del copies, src
    churn = None if args.no_churn else dnat_new_flows(m, o, flows, t0 + 1000, dev, torch)
    return {"cpu_baseline": cpu,
            "new_flows": churn,
            "workload": "NAT forward, established flows: 64B pkts (64B slots), "
                        "%d pkts per call over %d mappings" % (n, nflow),
            "pkts": n, "ms_per_step": round(ms, 4),
            "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": _roof(130, n, ms, "dnat"),
            "note": "per call: fused lookup+rewrite kernel (64 B slab), "
                    "4-byte miss count read back",
            "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                      if parity else "MISMATCH"}


def dnat_new_flows(m, o, flows, t0, dev, torch, nb=20, bn=1 << 16, frac=0.01):
    """NAT with a steady rate of new flows: nb forward batches of bn 64 B
    packets, `frac` of them from flows never seen before (each needs the
    host's port search), the rest from the established mappings. Per call:
    the fused pass, the new flows walked on the host in packet order, only
    the changed map words and entries sent to the device, then their
    packets stamped. Every batch checked against the oracle run on the same
    sequence (gates and frame bytes)."""
    from bess_amd import packets as P
    rng = np.random.default_rng(29)
    nnew = int(bn * frac)
    batches = []
    for b in range(nb):
        x = flows[rng.integers(0, flows.shape[0], bn)].copy()
        _, _, fresh = P.em_workload(16, nnew, seed=0x5EED, pkt_seed=1000 + b)
        zero = (fresh[:, 34] == 0) & (fresh[:, 35] == 0)
        fresh[zero, 35] = 1
        x[rng.choice(bn, nnew, replace=False)] = fresh
        batches.append(x)
    d = [torch.from_numpy(x.reshape(-1).copy()).to(dev) for x in batches]
    g = torch.empty(bn, dtype=torch.int16, device=dev)
    outs = []
    torch.cuda.synchronize()
    ms = []
    for b in range(nb):
        t = time.perf_counter()
        m.process_device(d[b], 64, bn, g, t0 + b)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t) * 1e3)
        outs.append((g.cpu().numpy().view(np.uint16).copy(), d[b].cpu().numpy()))
    ok = True
    for b in range(nb):
        ref = batches[b].copy()
        want = o.process(ref, 64, bn, 0, t0 + b)
        ok &= bool((outs[b][0] == want).all() and (outs[b][1] == ref.reshape(-1)).all())
    med = float(np.median(ms))
    return {"workload": "%d batches of %d 64B pkts, %.0f%% new flows each "
                        "(%d), the rest established; map grows from %d"
                        % (nb, bn, frac * 100, nnew, flows.shape[0]),
            "ms_per_batch_median": round(med, 4),
            "ms_per_batch_max": round(max(ms), 4),
            "Mpps": round(bn / (med * 1e-3) / 1e6, 1),
            "timing": "host wall per synchronous call (fused pass, host walk of "
                      "the new flows, word-level map update, stamp pass)",
            "parity": "bit-exact vs oracle, all batches" if ok else "MISMATCH"}


def run_wm(args, dev, torch):
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    from oracle import oracle as O
    n0, rep = 1 << 20, 8
    n = n0 * rep
    # IMIX frames (60/590/1514 B, 7:4:1) in 2 KB slots; the classifier
    # reads only each frame's header line. 1M distinct frames generated on
    # the host, the 16 GB device slab holds them 8 times over.
    rk, rm, prio, gates, frames, flen = P.wm_workload(100000, n0, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    # parity: oracle WildcardMatch on the first 64K frames
    L = O.lib()
    ow = L.or_wm_new()
    for off, size in P.FIVE_TUPLE:
        L.or_wm_add_field(ow, off, size, None, 0)
    L.or_wm_init_done(ow)
    kb = np.zeros(64, np.uint8)
    mb = np.zeros(64, np.uint8)
    for k, m, p, g in zip(rk, rm, prio, gates):
        kb[:16] = k
        mb[:16] = m
        L.or_wm_add(ow, kb.ctypes.data, mb.ctypes.data, int(p), int(g))
    ns = 1 << 16
    sample = np.ascontiguousarray(frames[:ns])
    want = np.zeros(ns, np.uint16)
    L.or_wm_process(ow, sample.ctypes.data, 2048, ns, 8192, want.ctypes.data)

    # the run-time compiled kernel of this rule set (bg_wm_jit.cc): the
    # product's launch once ready; compiled on a background thread
    from bess_amd import _lib as LB
    tj = time.time()
    t.jit_wait()
    jit_s = time.time() - tj

    def timed(slab, stride, gates, flags=0):
        with LB.kernel_paths(flags):
            clock_settle(args, torch, lambda: t.classify(slab, stride, n, 8192, gates))
            for _ in range(args.warmup):
                t.classify(slab, stride, n, 8192, gates)
            torch.cuda.synchronize()
            timer = Timer(torch)
            k = leg_steps(args)
            timer.start()
            for _ in range(k):
                t.classify(slab, stride, n, 8192, gates)
            return timer.stop_ms() / k

    def aot_check(slab, stride, gates, g_jit, flags=LB.BG_PATH_WM_NO_JIT):
        """another form of the kernel (default: the ahead-of-time one): same
        gates, its time"""
        with LB.kernel_paths(flags):
            t.classify(slab, stride, n, 8192, gates)
            torch.cuda.synchronize()
        same = bool((gates.cpu().numpy().view(np.uint16)[:n0] == g_jit).all())
        return same, timed(slab, stride, gates, flags)

    def check(gates_t):
        got = gates_t.cpu().numpy().view(np.uint16)
        return bool((got[:ns] == want).all() and
                    (got.reshape(rep, n0) == got[:n0]).all()), got[:n0]

    nan = float("nan")
    parity, ms2k, g2k, aot2k, aot_h = True, nan, None, nan, nan
    placement = None
    if args.wm_layout != "slab":  # the frames in 2 KB slots
        d0 = torch.from_numpy(frames.reshape(-1)).to(dev)
        dg = torch.empty(n, dtype=torch.int16, device=dev)
        d, placement = placed_slab(
            lambda: d0.repeat(rep),
            lambda sl: probe_ms(lambda: t.classify(sl, 2048, n, 8192, dg), torch), torch)
        del d0
        t.classify(d, 2048, n, 8192, dg)
        torch.cuda.synchronize()
        parity, g2k = check(dg)
        ms2k = timed(d, 2048, dg)
        same2k, aot2k = aot_check(d, 2048, dg, g2k)
        parity = parity and same2k
        del d, dg
    gbs2k = EM_BYTES_PER_PKT * n / (ms2k * 1e-3) / 1e9
    # The same packets' header lines in a dense 64 B slab: the layout the
    # north star asks for ("batches laid out for coalesced HBM reads of
    # header bytes"), which the host ingress (bg_pipe) stages anyway.
    ms, parity_h = nan, True
    if args.wm_layout != "2k":
        h0 = torch.from_numpy(np.ascontiguousarray(frames[:, :64]).reshape(-1)).to(dev)
        hs = h0.repeat(rep)
        del h0
        dgh = torch.empty(n, dtype=torch.int16, device=dev)
        t.classify(hs, 64, n, 8192, dgh)
        torch.cuda.synchronize()
        parity_h, gh = check(dgh)
        if g2k is not None:
            parity_h = parity_h and bool((gh == g2k).all())
        ms = timed(hs, 64, dgh)
        same_h, aot_h = aot_check(hs, 64, dgh, gh)
        parity_h = parity_h and same_h
        del hs, dgh
    mpps = n / (ms * 1e-3) / 1e6
    gbs = EM_BYTES_PER_PKT * n / (ms * 1e-3) / 1e9
    nbytes, in_lds = t.table_info()
    out = {"workload": "C4: 100K-rule WildcardMatch over 8 masks (tuple-space,"
                       " priority ties), 5-tuple, IMIX frames' header lines in "
                       "a dense 64B slab (beside: the frames in 2KB slots)",
           "pkts": n, "ms_per_step": round(ms, 4), "Mpps": round(mpps, 1),
           "table_bytes": nbytes,
           "table_in_lds": {0: "no (L2/MALL)", 1: "whole table",
                            2: "key filter (table in L2/MALL)",
                            3: "tag words (keys/values in L2/MALL)"}[int(in_lds)],
           "direct_tuples": t.direct_tuples(),
           "kernel": "run-time compiled for this rule set's shape (bg_wm_jit.cc, "
                     "hiprtc, %.2f s on a background thread); ahead-of-time "
                     "kernel beside" % jit_s,
           "ahead_of_time": {"ms_per_step": round(aot_h, 4),
                             "slots_2k_ms_per_step": round(aot2k, 4),
                             "same_gates": bool(parity and parity_h)},
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "traffic": traffic_gbs("wm", ms),
                        "traffic_bytes_per_launch": load_traffic("wm")},
           "parity": "bit-exact vs oracle on 64K-pkt samples of both layouts; "
                     "header-slab gates == 2KB-slot gates on all %d pkts" % n0
                     if parity and parity_h else "MISMATCH",
           "slots_2k": {"ms_per_step": round(ms2k, 4), "placement": placement,
                        "Mpps": round(n / (ms2k * 1e-3) / 1e6, 1),
                        "roofline": {"bound": "hbm", "achieved": round(gbs2k, 1),
                                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(gbs2k / HBM_PEAK_GBS, 4),
                                     "traffic": traffic_gbs("wm2k", ms2k),
                                     "traffic_bytes_per_launch": load_traffic("wm2k")},
                        "measured_ceiling": shape_ceiling("s2k32", n, ms2k)}}
    if not args.no_cpu:
        cn = 1 << 16
        g = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: L.or_wm_bench(ow, sample.ctypes.data, 2048, cn,
                                           8192, g.ctypes.data, nt, reps),
            cn, args.cpu_seconds / 2)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d IMIX frames x reps in 2048B slots, 100K-rule "
                          "WildcardMatch (8 CuckooMap tuples, CRC32C)" % cn)
    L.or_wm_free(ow)
    return out


def oracle_em_bulk(keys, gates):
    """the oracle ExactMatch (CuckooMap restatement) holding every rule"""
    from bess_amd import packets as P
    from oracle import oracle as O
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates, dtype=np.uint16)
    rc = L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data)
    if rc:
        raise RuntimeError("oracle rule insert failed: %d" % rc)
    return em


def c5_parity(keys, gates, sample, got):
    from oracle import oracle as O
    L = O.lib()
    em = oracle_em_bulk(keys, gates)
    want = np.zeros(sample.shape[0], np.uint16)
    L.or_em_process(em, sample.ctypes.data, 64, sample.shape[0], 8192,
                    want.ctypes.data)
    L.or_em_free(em)
    return bool((got == want).all())


def run_c5(args, dev, torch):
    """C5 on one GPU: 1M-rule 5-tuple ExactMatch (table in HBM / MALL, not
    LDS), 16M resident 64 B packets. The multi-GPU form (run_c5_multi) is
    in the N > 1 line; here the 8-way partition build is timed on the host
    as one rank of 8 runs it (inserting only its partition's rules)."""
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    from oracle import oracle as O
    n, nr = 16 << 20, 1 << 20
    keys, gates, frames = P.em_workload(nr, n, seed=0xC5, pkt_seed=0xC55)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    sample = np.ascontiguousarray(frames[:1 << 18])
    del frames
    dg = torch.empty(n, dtype=torch.int16, device=dev)
    t = F.EmTable(P.em_fields_5tuple())
    t0 = time.perf_counter()
    t.add_many(keys, gates)
    t.sync(dev.index)
    build_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    t8 = F.EmTable(P.em_fields_5tuple())
    t8.add_many(keys, gates, part=0, nparts=8)
    pb = t8.plan_count(8, t8.part_count(0, 8))
    part = t8.build_part(0, pb)
    part_s = time.perf_counter() - t0
    del part, t8
    t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    ns = sample.shape[0]
    parity = c5_parity(keys, gates, sample, dg[:ns].cpu().numpy().view(np.uint16))
    clock_settle(args, torch, lambda: t.classify(d, 64, n, 8192, dg))
    for _ in range(args.warmup):
        t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    timer = Timer(torch)
    k = leg_steps(args)
    timer.start()
    for _ in range(k):
        t.classify(d, 64, n, 8192, dg)
    ms = timer.stop_ms() / k
    mpps = n / (ms * 1e-3) / 1e6
    gbs = EM_BYTES_PER_PKT * n / (ms * 1e-3) / 1e9
    nbytes, in_lds = t.table_info()
    out = {"workload": "C5 (1 GPU): 64B pkts, 1M-rule 5-tuple ExactMatch, "
                       "16M resident pkts, table in HBM/MALL",
           "pkts": n, "rules": nr, "ms_per_step": round(ms, 4),
           "Mpps": round(mpps, 1), "table_bytes": nbytes,
           "host_table_build_s": round(build_s, 2),
           "host_partition_build_s_per_rank_of_8": round(part_s, 3),
           "partition_bytes": pb,
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "traffic": traffic_gbs("c5", ms),
                        "traffic_bytes_per_launch": load_traffic("c5"),
                        "traffic_note": "counts the table's random reads the "
                                        "Infinity Cache serves (r03 calibration)"},
           # no measured ceiling: the kernel outruns both random-probe
           # shapes of scripts/hbm_probe.hip, even rnd36s (its own whole-line
           # stream plus the same random tag and key reads; 0.400 ms for
           # 16 M on the r04 box against the kernel's 0.380,
           # profiles/r04_calibration.json), so neither bounds it
           "measured_ceiling": None,
           "parity": "bit-exact vs oracle on 256K-pkt sample" if parity
                     else "MISMATCH"}
    if not args.no_cpu:
        L = O.lib()
        em = oracle_em_bulk(keys, gates)
        cn = ns
        snb = np.zeros((cn, 2624), np.uint8)
        snb[:, 512:512 + 64] = sample
        og = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: L.or_em_bench(em, snb.ctypes.data + 512, 2624, cn,
                                           8192, og.ctypes.data, nt, reps),
            cn, args.cpu_seconds / 3)
        L.or_em_free(em)
        out["cpu_baseline"] = cpu_baseline(
            res, threads, "%d 64B pkts x reps in snbuf layout, 1M-rule 5-tuple "
                          "ExactMatch (CuckooMap/CRC32C restated)" % cn)
    return out


def _agree(ok, dist, torch, dev):
    """True when the step succeeded on every rank: a rank that failed says
    so before the others enter a collective it would never join"""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def run_c5_multi(args, rank, world, dev, torch, dist):
    """C5 at N = world GPUs: 1M rules sharded over the ranks (rank r inserts
    only partition r's rules; all-reduce MAX of the partition sizes fixes
    the layout; each rank builds its partition; one all-gather of the
    partition images over RCCL/xGMI assembles the replicated table), then
    every rank classifies its own 16M packets through the 1M-rule table.
    The collective is the C ABI's own (bg_comm_init_rank + bg_em_allgather,
    what a bessd calls): torch.distributed carries only the communicator's
    128-byte id and the timing reductions, never the table."""
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    n, nr = args.pkts, args.c5_rules
    keys, gates, frames = P.em_workload(nr, n, seed=0xC5,
                                        pkt_seed=0xC55 + 7919 * rank)
    d = torch.from_numpy(frames.reshape(-1)).to(dev)
    sample = np.ascontiguousarray(frames[:1 << 18])
    del frames
    dg = torch.empty(n, dtype=torch.int16, device=dev)
    t = F.EmTable(P.em_fields_5tuple())
    dist.barrier()
    t0 = time.perf_counter()
    err = None
    try:
        t.add_many(keys, gates, part=rank, nparts=world)
    except Exception as e:
        err = e
    if not _agree(err is None, dist, torch, dev):
        raise RuntimeError("C5 partition insert failed on a rank: %r" % (err,))
    insert_s = time.perf_counter() - t0
    held = len(t)
    comm = F.Comm.over_process_group(rank, world, dev.index, dist)
    dist.barrier()
    t0 = time.perf_counter()
    try:
        t.allgather(comm)
    except Exception as e:
        err = e
    if not _agree(err is None, dist, torch, dev):
        comm.close()
        raise RuntimeError("C5 all-gather failed on a rank: %r" % (err,))
    st = comm.last_stats()
    st["call_ms"] = (time.perf_counter() - t0) * 1e3
    t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    ns = sample.shape[0]
    parity = c5_parity(keys, gates, sample, dg[:ns].cpu().numpy().view(np.uint16))
    clock_settle(args, torch, lambda: t.classify(d, 64, n, 8192, dg))
    for _ in range(args.warmup):
        t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    timer = Timer(torch)
    dist.barrier()
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    timer.start()
    for _ in range(args.steps):
        t.classify(d, 64, n, 8192, dg)
    kern_ms = timer.stop_ms() / args.steps
    torch.cuda.synchronize()
    dist.barrier()
    wall = time.perf_counter() - w0
    per = torch.tensor([wall, kern_ms, insert_s * 1e3, st["build_ms"],
                        st["allgather_ms"], held, 1.0 if parity else 0.0,
                        st["allreduce_ms"], st["call_ms"]],
                       dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(per) for _ in range(world)]
    dist.all_gather(allr, per)
    allr = [x.tolist() for x in allr]
    wall = max(x[0] for x in allr)
    kern = max(x[1] for x in allr)
    gbs = EM_BYTES_PER_PKT * n / (kern * 1e-3) / 1e9
    nbytes, _ = t.table_info()
    return {"workload": "C5: 64B pkts, %d-rule 5-tuple ExactMatch sharded over %d "
                        "GPUs (RCCL all-gather of the partition images), %d "
                        "resident pkts per GPU" % (nr, world, n),
            "n_gpus": world, "rules": nr, "pkts_per_gpu": n,
            "value": round(n * world * args.steps / wall / 1e6, 1), "unit": "Mpps",
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "per_rank_Mpps": [round(n / (x[1] * 1e-3) / 1e6, 1) for x in allr],
            "rules_inserted_per_rank": [int(x[5]) for x in allr],
            "insert_ms_per_rank": [round(x[2], 1) for x in allr],
            "collective": "bg_em_allgather (C ABI, RCCL)",
            "part_build_ms": round(max(x[3] for x in allr), 2),
            "size_allreduce_ms": round(max(x[7] for x in allr), 3),
            "allgather_ms": round(max(x[4] for x in allr), 3),
            "allgather_call_ms": round(max(x[8] for x in allr), 3),
            "allgather_bytes": st["bytes"], "table_bytes": nbytes,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "per": "GPU (slowest rank's kernel)"},
            "parity": "bit-exact vs oracle on 256K pkts per rank"
                      if all(x[6] for x in allr) else "MISMATCH",
            "_comm": comm}


def run_c1(args):
    """C1 (bessctl/conf/samples/exactmatch.bess shape, CPU only): Source ->
    ExactMatch(1 rule, 5-tuple) -> Sink on the host, 60 B frames (64 B
    packets) from a pool of snbuf-like buffers, 32-packet batches, gate 0
    connected to the Sink, default DROP_GATE. The oracle restatement of the
    reference path (MakeKeys + CuckooMap::Find + EmitPacket's per-gate
    batches + Sink) is timed; no GPU (plumbing)."""
    from bess_amd import packets as P
    from oracle import oracle as O
    import ctypes as C
    L = O.lib()
    n = 1 << 18
    keys, gates, frames = P.em_workload(1, n, hit_frac=1.0, seed=0xC1)
    em = oracle_em_bulk(keys, np.zeros(1, np.uint16))
    snb = np.zeros((n, 2624), np.uint8)
    snb[:, 512:512 + 64] = frames
    og = np.zeros(n, np.uint16)
    sunk = C.c_uint64()
    threads, res = cpu_rate(
        lambda nt, reps: L.or_c1_bench(em, snb.ctypes.data + 512, 2624, n, 8192,
                                       1, og.ctypes.data, nt, reps,
                                       C.byref(sunk)),
        n, args.cpu_seconds / 3)
    L.or_c1_bench(em, snb.ctypes.data + 512, 2624, n, 8192, 1, og.ctypes.data,
                  1, 1, C.byref(sunk))
    L.or_em_free(em)
    ok = bool((og == 0).all() and sunk.value == n)
    return {"workload": "C1: Source -> ExactMatch(1 rule, 5-tuple) -> Sink on "
                        "CPU, 60B frames (64B pkts), 32-pkt batches",
            "Mpps": round(res[threads], 2), "unit": "Mpps",
            "cpu_baseline": cpu_baseline(
                res, threads, "%d 64B pkts x reps in snbuf layout; per batch: "
                              "MakeKeys, CuckooMap::Find, EmitPacket per-gate "
                              "batches, Sink" % n),
            "parity": "every packet to gate 0 and the sink" if ok else "MISMATCH"}


def run_table_only(args, rank, world):
    """--cpu-table-only: the C5 control path of an N-rank run on CPU (gloo):
    rank r inserts only partition r's rules, all-reduce MAX, build, all-gather
    of the partition images; rank 0 checks the gathered image is byte-equal
    to a single-process build of the whole rule set."""
    import torch.distributed as dist
    from bess_amd import dist as D
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    nr = args.c5_rules
    keys, gates, _ = P.em_workload(nr, 1, seed=0xC5)
    t = F.EmTable(P.em_fields_5tuple())
    t0 = time.perf_counter()
    t.add_many(keys, gates, part=rank, nparts=world)
    insert_ms = (time.perf_counter() - t0) * 1e3
    if world > 1:
        full, st = D.sharded_em_table(t, rank, world)
    else:
        pb = t.plan(1)
        full, st = t.build_part(0, pb), {"part_bytes": pb, "bytes": pb,
                                         "build_ms": 0.0, "allgather_ms": 0.0}
    same = None
    if rank == 0:
        ref = F.EmTable(P.em_fields_5tuple())
        ref.add_many(keys, gates)
        same = bool(np.array_equal(np.asarray(full), D.local_image(ref, world)))
    if rank == 0:
        print(json.dumps({
            "metric": "Mpps + %HBM-roofline, device-resident parse+match, "
                      "64B/1500B, 1/2/4/8 GPU", "value": None, "unit": "Mpps",
            "n_gpus": world, "mode": "cpu-table-only (gloo, no GPU)",
            "C5_table": {"rules": nr, "rules_inserted_rank0": len(t),
                         "insert_ms_rank0": round(insert_ms, 1),
                         "part_bytes": st["part_bytes"], "bytes": st["bytes"],
                         "part_build_ms": round(st["build_ms"], 2),
                         "allgather_ms": round(st["allgather_ms"], 3),
                         "image_equals_single_build": same}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if same in (None, True) else 1


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def main():
    args = parse()
    if args.lib:
        from bess_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # start the N ranks (one process per GPU) before anything touches a
        # GPU, and exit with their exit code
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node=%d" % args.gpus, "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__)]
        cmd += sys.argv[1:]
        log("bench.py: starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
        sys.exit(subprocess.call(cmd))
    world = int(env_world or "1")
    if world != args.gpus:
        log("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
        sys.exit(2)
    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_table_only:
        return run_table_only(args, rank, world)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # a bounded wait: a rank that died must not hold the others forever
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(minutes=5))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import bess_amd
    bess_amd.lib()  # fail loudly if the HIP library is missing

    only = {"cksum": lambda: run_cksum(args, dev, torch),
            "em1500": lambda: run_em1500(args, dev, torch),
            "wm": lambda: run_wm(args, dev, torch),
            "c5": lambda: run_c5(args, dev, torch),
            "ttl": lambda: run_update_ttl(args, dev, torch),
            "dnat": lambda: run_dnat(args, dev, torch),
            "rewrite": lambda: run_rewrite(args, dev, torch),
            "nat": lambda: run_static_nat(args, dev, torch),
            "iplookup": lambda: run_iplookup(args, dev, torch),
            "acl": lambda: run_acl(args, dev, torch),
            "hashlb": lambda: run_hashlb(args, dev, torch),
            "pipe": lambda: run_e2e_pipe(args, torch),
            "plugin": lambda: run_plugin_pipeline(args),
            "plugin_pool": lambda: run_plugin_pool(args),
            "c1": lambda: run_c1(args),
            "sweep": lambda: em_sweep(run_em(args, rank, world, dev, torch,
                                             dist), torch)}
    if args.only:
        log(json.dumps(only[args.only]()))
        return

    r = run_em(args, rank, world, dev, torch, dist)
    n_total = r["n"] * world
    ms_step = r["wall"] / args.steps * 1e3
    value = n_total * args.steps / r["wall"] / 1e6
    kern_ms = r["kern_ms"] / args.steps
    achieved = EM_BYTES_PER_PKT * r["n"] / (kern_ms * 1e-3) / 1e9
    out = {
        "metric": "Mpps + %HBM-roofline, device-resident parse+match, "
                  "64B/1500B, 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "Mpps", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "settle_ms": args.settle_ms,
        "settle": "untimed, before the warm-up: ~settle_ms of the headline's own "
                  "launch (it leaves the slab as it was)",
        "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded 5-tuple traffic, 50% rule hits)",
        "config": {"workload": "C2: 64B pkts (60B frames, 64B slots), %d-rule "
                               "5-tuple ExactMatch, %d resident pkts per GPU"
                               % (args.rules, r["n"]),
                   "rules": args.rules, "pkts_per_gpu": r["n"],
                   "slot_bytes": 64, "parallelism": "dp%d (packet shards)" % world,
                   "table": r["table"]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_gbs("em", kern_ms)
                     if args.rules == 1000 and r["n"] == 16 << 20 else None,
                     "traffic_bytes_per_launch": load_traffic("em")
                     if args.rules == 1000 and r["n"] == 16 << 20 else None,
                     "kernel": "em_slab_kernel",
                     "kernel_ms": round(kern_ms, 4),
                     "bytes_per_pkt": EM_BYTES_PER_PKT},
        "parity": "bit-exact vs oracle on 1M-pkt sample" if r["parity"]
                  else "MISMATCH",
        # the same memory traffic without the lookup (hbm_probe slab66)
        # the fastest measured shape that writes the gates (round 6: gates
        # held in LDS to the end; the reads alone are c2_read64)
        "measured_ceiling": shape_ceiling("c2_lds128", r["n"], kern_ms),
        "cpu_baseline": None,
    }
    comm = None  # C5's communicator (N > 1), closed before the process group
    if world > 1:
        del r
        torch.cuda.empty_cache()
        try:
            out["C5"] = run_c5_multi(args, rank, world, dev, torch, dist)
            comm = out["C5"].pop("_comm")
        except Exception as e:  # report, do not hide
            out["C5"] = "failed: %r" % (e,)
    def attempt(fn, *a):
        try:
            return fn(*a)
        except Exception as e:  # report, do not hide
            return "failed: %r" % (e,)

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_em(r["keys"], r["gates"],
                                              args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_extra:
        # Ordered by weight, lightest first: the driver's record keeps the
        # line's last ~8 KB, which then hold the SURVEY configs (C3, the
        # 1500 B match point, C4, C5), the batch sweep and the plugin legs.
        sweep = attempt(em_sweep, r, torch)
        out["modules_8f"] = {}
        for name, fn in (("HashLB", run_hashlb), ("ACL", run_acl),
                         ("IPLookup", run_iplookup),
                         ("UpdateTTL", run_update_ttl),
                         ("StaticNAT", run_static_nat),
                         ("NAT", run_dnat), ("Rewrite", run_rewrite)):
            out["modules_8f"][name] = attempt(fn, args, dev, torch)
        if not args.no_cpu:
            out["C1"] = attempt(run_c1, args)
        if not args.no_e2e:
            out["e2e_host"] = attempt(run_e2e_host, r, args, torch)
            out["e2e_pipe"] = attempt(run_e2e_pipe, args, torch)
            out["e2e_plugin"] = attempt(run_plugin_pipeline, args)
            out["e2e_plugin_pool"] = attempt(run_plugin_pool, args)
        out["batch_sweep_mpps"] = sweep
        out["extra_configs"] = {}
        for name, fn in (("C3", run_cksum), ("EM_1500B", run_em1500),
                         ("C4", run_wm), ("C5", run_c5)):
            out["extra_configs"][name] = attempt(fn, args, dev, torch)
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        if comm is not None:
            torch.cuda.synchronize()
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

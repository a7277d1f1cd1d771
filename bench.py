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

N > 1: every rank owns its own 16 M packets (weak scaling, no data-path
collective). The rule table is built sharded: rank r builds partition r of
the flow table and an RCCL all-gather over xGMI assembles the replicated
table on every GPU (the only collective; control path, timed separately).

Rank 0 prints ONE JSON line. Secondary configs (C3 checksum, C4 wildcard,
batch-size sweep) are measured at N = 1 only, as extra keys.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table
EM_BYTES_PER_PKT = 66  # 64 B header line read + 2 B gate written
CK_BYTES_PER_PKT = 1502  # 1496 B frame read + IP csum + L4 csum + gate (2 B each)


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
    ap.add_argument("--only", default="", help="cksum|wm|c5|hashlb|acl|iplookup|ttl|nat|dnat|pipe (profiling runs)")
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


def traffic_gbs(key, kernel_ms):
    """PMC bytes per launch / measured launch duration, in GB/s (same basis
    as roofline.achieved); None until profiles/ holds a PMC measurement."""
    b = load_traffic(key)
    return None if b is None else round(b / (kernel_ms * 1e-3) / 1e9, 1)


def em_setup(args, rank, world, dev, torch, dist):
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    t0 = time.time()
    # same rules on every rank, rank-specific packets
    keys, gates, frames = P.em_workload(args.rules, args.pkts, seed=0x5EED,
                                        pkt_seed=0x5EED + 7919 * rank)
    log("[rank %d] workload generated in %.1fs" % (rank, time.time() - t0))
    d_frames = torch.from_numpy(frames.reshape(-1)).to(dev)
    del frames
    d_gates = torch.empty(args.pkts, dtype=torch.int16, device=dev)
    t = F.EmTable(P.em_fields_5tuple())
    t0 = time.time()
    t.add_many(keys, gates)
    log("[rank %d] %d rules inserted in %.1fs" % (rank, len(t), time.time() - t0))
    table = {"rules": len(t)}
    if world > 1:
        # sharded build + RCCL all-gather of the partition images
        from bess_amd import dist as D
        dist.barrier()
        _, st = D.sharded_em_table(t, rank, world, device=dev)
        table["allgather_ms"] = round(st["allgather_ms"], 3)
        table["allgather_bytes"] = st["bytes"]
        table["part_build_ms"] = round(st["build_ms"], 2)
    else:
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
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    sizes = [s for _, s in P.FIVE_TUPLE]
    pos = np.cumsum([0] + sizes)
    ptrs = (C.c_void_p * 5)()
    lens = (C.c_size_t * 5)(*sizes)
    keys = np.ascontiguousarray(keys)
    for k, g in zip(keys, gates):
        for j in range(5):
            ptrs[j] = k.ctypes.data + int(pos[j])
        L.or_em_add_rule(em, int(g), ptrs, lens, 5, None, 0)
    want = np.zeros(n, np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, n, 8192, want.ctypes.data)
    L.or_em_free(em)
    return bool((got == want).all())


def cpu_rate(bench, n, seconds):
    """Time the oracle's pthread bench driver `bench(nthreads, reps)` (returns
    seconds) at 1 thread and at T = min(16, usable cores) threads; about
    `seconds` of CPU work in total. Returns (T, {threads: Mpps})."""
    from oracle import oracle as O
    threads = max(1, min(16, O.lib().or_num_cpus()))
    res = {}
    for nt in sorted({1, threads}):
        t1 = bench(nt, 1)
        reps = max(1, int(seconds / 2 / max(t1, 1e-6)))
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
    threads = max(1, min(16, L.or_num_cpus()))
    res = {}
    for nt in sorted({1, threads}):
        t1 = L.or_em_bench(em, base, 2624, n, 8192, out.ctypes.data, nt, 1)
        reps = max(1, int(seconds / 2 / max(t1, 1e-6)))
        dt = L.or_em_bench(em, base, 2624, n, 8192, out.ctypes.data, nt, reps)
        res[nt] = n * reps / dt / 1e6
    L.or_em_free(em)
    return {"value": round(res[threads], 2), "unit": "Mpps", "cores": threads,
            "kind": "port",
            "single_core_mpps": round(res[1], 2),
            "sample": "%d 64B pkts x reps, 1K-rule 5-tuple ExactMatch, snbuf "
                      "layout (2624 B stride), 32-pkt batches, %d pinned "
                      "threads" % (n, threads)}


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
              sees);
      graph:  the 512 launches captured in a HIP graph and replayed (no
              host cost; the runtime may overlap independent launches)."""
    t, d_frames, d_gates = r["t"], r["d_frames"], r["d_gates"]
    out = {"stream": {}, "graph": {}}
    s = torch.cuda.Stream()
    nl = 512

    import ctypes as C
    from bess_amd import lib
    classify = lib().bg_em_classify
    fp, gp, sp = d_frames.data_ptr(), d_gates.data_ptr(), C.c_void_p(s.cuda_stream)

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
    for _ in range(args.warmup):  # recompute is idempotent
        F.cksum(d, 2048, n, 3, False, None, l4g)
    torch.cuda.synchronize()
    timer = Timer(torch)
    torch.cuda.synchronize()
    timer.start()
    for _ in range(args.steps):
        F.cksum(d, 2048, n, 3, False, None, l4g)
    ms = timer.stop_ms() / args.steps
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
        out["cpu_baseline"] = {
            "value": round(res[threads], 2), "unit": "Mpps", "cores": threads,
            "kind": "port", "single_core_mpps": round(res[1], 2),
            "sample": "%d 1496B frames x reps in 2048B slots, IPChecksum->"
                      "L4Checksum (AVX2/adc CalculateSum restated)" % cn}
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
            "Mpps_by_batch": res}


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
    em = {}
    for batch in (4096, 65536):
        p = Pipe(m, batch=batch, depth=4)
        em["parity_batch%d" % batch] = bool((p.run(heads) == want).all())
        p.close()
        rates = {}
        for th in (1, 4, 16):
            rates[str(th)] = _pipe_rate(
                lambda: Pipe(m, batch=batch, depth=4), heads, None, th,
                reps=2 if th == 1 else 4)
        em["Mpps_by_threads_batch%d" % batch] = rates
    out["ExactMatch_64B"] = em
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
    for th in (1, 4, 16):
        rates[str(th)] = _pipe_rate(
            lambda: Pipe(mk, batch=8192, depth=4, span=1504), heads, lens, th,
            reps=4)
    ck["Mpps_by_threads_batch8192"] = rates
    ck["bytes_per_pkt_pcie"] = {"h2d": 1504, "d2h": 130}
    out["L4Checksum_1500B"] = ck
    return out


def _time_steps(step, args, torch):
    """warmup, then ms per launch over args.steps launches (HIP events on
    the launching stream)"""
    for _ in range(max(3, args.warmup // 4)):
        step()
    torch.cuda.synchronize()
    timer = Timer(torch)
    reps = 10
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
        ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
        out[name] = {"ms_per_step": round(ms, 4),
                     "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
                     "roofline": _roof(EM_BYTES_PER_PKT, n, ms,
                                       "hashlb" if name == "l4" else None),
                     "parity": "bit-exact vs oracle on %d pkts" % k
                               if parity else "MISMATCH"}
        if name == "l4" and not args.no_cpu:
            cn = 1 << 18
            snb = _snbuf_sample(frames, cn)
            og = np.zeros(cn, np.uint16)
            gt = np.array(o.gates_, np.uint16)
            L = OM.mlib()
            threads, res = cpu_rate(
                lambda nt, reps: L.or_hashlb_bench(
                    o.mode, None, 0, gt.ctypes.data, 8, snb.ctypes.data + 512,
                    2624, cn, og.ctypes.data, nt, reps), cn, args.cpu_seconds / 3)
            out[name]["cpu_baseline"] = {
                "value": round(res[threads], 2), "unit": "Mpps",
                "cores": threads, "kind": "port",
                "single_core_mpps": round(res[1], 2),
                "sample": "%d 64B pkts x reps in snbuf layout, HashLB l4 "
                          "(SSE4.2 CRC32C)" % cn}
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
        ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
        e = {"ms_per_step": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
             "roofline": _roof(EM_BYTES_PER_PKT, n, ms, "acl"),
             "parity": "bit-exact vs oracle on %d pkts" % k if parity else "MISMATCH"}
        if not args.no_cpu:
            cn = 1 << 16
            snb = _snbuf_sample(frames, cn)
            threads, res = cpu_rate(
                lambda nt, reps: o.bench(snb.ctypes.data + 512, 2624, cn, nt, reps),
                cn, args.cpu_seconds / 4)
            e["cpu_baseline"] = {
                "value": round(res[threads], 2), "unit": "Mpps", "cores": threads,
                "kind": "port", "single_core_mpps": round(res[1], 2),
                "sample": "%d 64B pkts x reps in snbuf layout, %d-rule ACL" % (cn, nr)}
        out["rules_%d" % nr] = e
        del d
    return out


def run_iplookup(args, dev, torch):
    """IPLookup (core/modules/ip_lookup.cc) on the C2 slab: 16M 64 B packets,
    10K routes (/8../24, 5 % /25../32, nested), half the destinations inside
    a route; DIR-24-8 tables (32 MB tbl24) in HBM/MALL"""
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
    ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
    out = {"workload": "IPLookup: 64B pkts (64B slots), %d resident pkts, 10K "
                       "routes, DIR-24-8" % n, "pkts": n, "routes": len(o.rules),
           "ms_per_step": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
           "roofline": _roof(EM_BYTES_PER_PKT, n, ms, "iplookup"),
           "parity": "bit-exact vs oracle on %d pkts" % k if parity else "MISMATCH"}
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
    return {"workload": "UpdateTTL: 64B pkts (64B slots), %d resident pkts, in "
                        "place" % n, "pkts": n, "ms_per_step": round(ms, 4),
            "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": _roof(130, n, ms, "ttl"),
            "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                      if parity else "MISMATCH"}


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
    pairs scanned). Bytes/pkt: 64 B line read + 64 B written back + 2 B
    gate = 130."""
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
    ms = _time_steps(lambda: m.process_device(d, 64, n, g), args, torch)
    return {"workload": "StaticNAT forward: 64B pkts (64B slots), %d resident "
                        "pkts, 16 pairs, 50%% translated, in place" % n,
            "pkts": n, "ms_per_step": round(ms, 4),
            "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": _roof(130, n, ms, "nat"),
            "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                      if parity else "MISMATCH"}


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
    timer = Timer(torch)
    timer.start()
    for i in range(reps):
        m.process_device(copies[i + 1], 64, n, g, t0 + 2 + i)
    ms = timer.stop_ms() / reps
    return {"workload": "NAT forward, established flows: 64B pkts (64B slots), "
                        "%d pkts per call over %d mappings" % (n, nflow),
            "pkts": n, "ms_per_step": round(ms, 4),
            "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": _roof(130, n, ms, "dnat"),
            "note": "per call: fused lookup+rewrite kernel (64 B slab), "
                    "4-byte miss count read back",
            "parity": "bit-exact (gates + frame bytes) vs oracle on %d pkts" % k
                      if parity else "MISMATCH"}


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
    d0 = torch.from_numpy(frames.reshape(-1)).to(dev)
    d = d0.repeat(rep)
    del d0
    dg = torch.empty(n, dtype=torch.int16, device=dev)
    t.classify(d, 2048, n, 8192, dg)
    torch.cuda.synchronize()
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
    got = dg.cpu().numpy().view(np.uint16)
    parity = bool((got[:ns] == want).all() and
                  (got.reshape(rep, n0) == got[:n0]).all())
    for _ in range(args.warmup):
        t.classify(d, 2048, n, 8192, dg)
    torch.cuda.synchronize()
    timer = Timer(torch)
    timer.start()
    for _ in range(args.steps):
        t.classify(d, 2048, n, 8192, dg)
    ms = timer.stop_ms() / args.steps
    mpps = n / (ms * 1e-3) / 1e6
    gbs = EM_BYTES_PER_PKT * n / (ms * 1e-3) / 1e9
    nbytes, in_lds = t.table_info()
    out = {"workload": "C4: 100K-rule WildcardMatch over 8 masks (tuple-space,"
                       " priority ties), 5-tuple, header lines of IMIX frames "
                       "in 2KB slots",
           "pkts": n, "ms_per_step": round(ms, 4), "Mpps": round(mpps, 1),
           "table_bytes": nbytes,
           "table_in_lds": {0: "no (L2/MALL)", 1: "whole table",
                            2: "key filter (table in L2/MALL)",
                            3: "tag words (keys/values in L2/MALL)"}[int(in_lds)],
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "traffic": traffic_gbs("wm", ms),
                        "traffic_bytes_per_launch": load_traffic("wm")},
           "parity": "bit-exact vs oracle on 64K-pkt sample" if parity
                     else "MISMATCH"}
    if not args.no_cpu:
        cn = 1 << 16
        g = np.zeros(cn, np.uint16)
        threads, res = cpu_rate(
            lambda nt, reps: L.or_wm_bench(ow, sample.ctypes.data, 2048, cn,
                                           8192, g.ctypes.data, nt, reps),
            cn, args.cpu_seconds / 2)
        out["cpu_baseline"] = {
            "value": round(res[threads], 2), "unit": "Mpps", "cores": threads,
            "kind": "port", "single_core_mpps": round(res[1], 2),
            "sample": "%d IMIX frames x reps in 2048B slots, 100K-rule "
                      "WildcardMatch (8 CuckooMap tuples, CRC32C)" % cn}
    L.or_wm_free(ow)
    return out


def run_c5(args, dev, torch):
    """C5 on one GPU: 1M-rule 5-tuple ExactMatch (table in HBM / MALL, not
    LDS), 16M resident 64 B packets. The multi-GPU form builds the table
    sharded and all-gathers it (dist.sharded_em_table); here the 8-way
    partition build is timed on the host as it would run per rank."""
    from bess_amd import flowtable as F
    from bess_amd import packets as P
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
    pb = t.plan(8)
    part = t.build_part(0, pb)
    part_s = time.perf_counter() - t0
    del part
    t.sync(dev.index)  # back to the single-device image
    t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    # parity on the first 256K packets
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
    ns = sample.shape[0]
    want = np.zeros(ns, np.uint16)
    L.or_em_process(em, sample.ctypes.data, 64, ns, 8192, want.ctypes.data)
    L.or_em_free(em)
    parity = bool((dg[:ns].cpu().numpy().view(np.uint16) == want).all())
    for _ in range(args.warmup):
        t.classify(d, 64, n, 8192, dg)
    torch.cuda.synchronize()
    timer = Timer(torch)
    timer.start()
    for _ in range(args.steps):
        t.classify(d, 64, n, 8192, dg)
    ms = timer.stop_ms() / args.steps
    mpps = n / (ms * 1e-3) / 1e6
    gbs = EM_BYTES_PER_PKT * n / (ms * 1e-3) / 1e9
    nbytes, in_lds = t.table_info()
    return {"workload": "C5 (1 GPU): 64B pkts, 1M-rule 5-tuple ExactMatch, "
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
                         "traffic_bytes_per_launch": load_traffic("c5")},
            "parity": "bit-exact vs oracle on 256K-pkt sample" if parity
                      else "MISMATCH"}


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import bess_amd
    bess_amd.lib()  # fail loudly if the HIP library is missing

    if args.only == "cksum":
        log(json.dumps(run_cksum(args, dev, torch)))
        return
    if args.only == "wm":
        log(json.dumps(run_wm(args, dev, torch)))
        return
    if args.only == "c5":
        log(json.dumps(run_c5(args, dev, torch)))
        return
    if args.only == "ttl":
        log(json.dumps(run_update_ttl(args, dev, torch)))
        return
    if args.only == "dnat":
        log(json.dumps(run_dnat(args, dev, torch)))
        return
    if args.only == "nat":
        log(json.dumps(run_static_nat(args, dev, torch)))
        return
    if args.only == "iplookup":
        log(json.dumps(run_iplookup(args, dev, torch)))
        return
    if args.only == "acl":
        log(json.dumps(run_acl(args, dev, torch)))
        return
    if args.only == "hashlb":
        log(json.dumps(run_hashlb(args, dev, torch)))
        return
    if args.only == "pipe":
        log(json.dumps(run_e2e_pipe(args, torch)))
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
        "steps": args.steps, "warmup": args.warmup,
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
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_extra:
        try:
            out["batch_sweep_mpps"] = em_sweep(r, torch)
        except Exception as e:  # report, do not hide
            out["batch_sweep_mpps"] = "failed: %r" % (e,)
        out["extra_configs"] = {}
        if not args.no_e2e:
            try:
                out["e2e_host"] = run_e2e_host(r, args, torch)
            except Exception as e:
                out["e2e_host"] = "failed: %r" % (e,)
            try:
                out["e2e_pipe"] = run_e2e_pipe(args, torch)
            except Exception as e:
                out["e2e_pipe"] = "failed: %r" % (e,)
        for name, fn in (("C3", run_cksum), ("C4", run_wm), ("C5", run_c5),
                         ("HashLB", run_hashlb), ("ACL", run_acl),
                         ("IPLookup", run_iplookup),
                         ("UpdateTTL", run_update_ttl),
                         ("StaticNAT", run_static_nat),
                         ("NAT", run_dnat)):
            try:
                out["extra_configs"][name] = fn(args, dev, torch)
            except Exception as e:
                out["extra_configs"][name] = "failed: %r" % (e,)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_em(r["keys"], r["gates"],
                                              args.cpu_seconds)
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

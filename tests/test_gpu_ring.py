"""The persistent classify kernel (bg_ring, em_ring_kernel): batches of the
sizes BESS hands a module (32 ... 4096 packets, ragged tails) through one
running kernel, bit-exact against the oracle; idle exit and relaunch; the
table snapshot; a 1M-rule table probed in L2."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


def oracle_gates(keys, gates, frames, default_gate=8192):
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates, dtype=np.uint16)
    assert L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data) == 0
    want = np.zeros(len(frames), np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, len(frames), default_gate,
                    want.ctypes.data)
    L.or_em_free(em)
    return want


@pytest.mark.parametrize("n_rules", [1000, 1 << 20])
def test_ring_batches_vs_oracle(n_rules):
    n = 1 << 18
    keys, gates, frames = P.em_workload(n_rules, n, seed=n_rules, pkt_seed=3)
    want = oracle_gates(keys, gates, frames)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    ring = F.Ring(t, slots=256)
    for burst in (32, 100, 4096):
        dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
        ring.run(d, 64, n, burst, 8192, dg)
        torch.cuda.synchronize()
        assert (dg.cpu().numpy().view(np.uint16) == want).all(), burst
    # individual tickets, out-of-order waits, a 1-packet batch
    dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
    tickets = [ring.submit(d, 64, 1, 8192, dg, offset=0)]
    tickets += [ring.submit(d, 64, 32, 8192, dg, offset=1 + 32 * i) for i in range(50)]
    ring.wait(tickets[-1])
    ring.wait(tickets[0])
    assert ring.completed() >= tickets[-1] + 1
    got = dg[:1 + 32 * 50].cpu().numpy().view(np.uint16)
    assert (got == want[:1 + 32 * 50]).all()
    launches, blocks = ring.info()
    assert launches >= 1 and blocks > 0
    ring.close()


def test_ring_idle_exit_relaunch_and_snapshot():
    n = 1 << 14
    keys, gates, frames = P.em_workload(1000, n, seed=5)
    want = oracle_gates(keys, gates, frames)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    ring = F.Ring(t, slots=64, idle_us=2000)
    dg = torch.zeros(n, dtype=torch.int16, device="cuda")
    ring.run(d, 64, n, 256, 8192, dg)
    assert (dg.cpu().numpy().view(np.uint16) == want).all()
    time.sleep(0.05)  # > idle: the grid has stopped itself
    t.clear()  # a rule change: the ring keeps its snapshot (and memory)
    t.sync(0)
    dg.zero_()
    ring.run(d, 64, n, 512, 8192, dg)
    assert (dg.cpu().numpy().view(np.uint16) == want).all()
    launches, _ = ring.info()
    assert launches >= 2
    ring.close()
    # a new ring sees the cleared table
    ring = F.Ring(t, slots=64)
    ring.run(d, 64, n, 512, 8192, dg)
    assert (dg.cpu().numpy().view(np.uint16) == 8192).all()
    ring.close()


@pytest.mark.parametrize("host_desc", [False, True])
@pytest.mark.parametrize("lanes,threads", [(4, 4), (16, 16), (16, 3)])
def test_ring_submission_lanes_vs_oracle(lanes, threads, host_desc):
    """several worker threads, each on its own submission lane of one
    running kernel, 32-packet batches (and ragged 100-packet ones): every
    gate as the oracle's; an idle exit in between relaunches for all lanes.
    Both descriptor homes: device memory written by the host (the default
    where the BAR maps it) and pinned host memory (BG_PATH_RING_HOST_DESC)"""
    from bess_amd._lib import kernel_paths, BG_PATH_RING_HOST_DESC
    with kernel_paths(BG_PATH_RING_HOST_DESC if host_desc else 0):
        _ring_submission_lanes(lanes, threads, host_desc)


def _ring_submission_lanes(lanes, threads, host_desc):
    n = 1 << 18
    keys, gates, frames = P.em_workload(1000, n, seed=lanes, pkt_seed=9)
    want = oracle_gates(keys, gates, frames)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    ring = F.Ring(t, slots=512, lanes=lanes, idle_us=3000)
    if host_desc:
        assert not ring.desc_in_device()
    for burst in (32, 100):
        dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
        ring.run_lanes(d, 64, n, burst, 8192, dg, threads)
        torch.cuda.synchronize()
        assert (dg.cpu().numpy().view(np.uint16) == want).all(), burst
        time.sleep(0.02)  # idle: the grid stops; the next run relaunches it
    launches, _ = ring.info()
    assert launches >= 2
    # tickets count per lane
    for lane in range(min(lanes, 3)):
        tk = ring.submit(d, 64, 32, 8192, dg, offset=32 * lane, lane=lane)
        ring.wait(tk, lane=lane)
        assert ring.completed(lane=lane) == tk + 1
    ring.close()


def test_ring_mixed_runs_vs_oracle():
    """a workgroup takes the published tickets of its claimed range as one
    run (em_ring_kernel): consecutive tickets of ragged sizes (0 to 300
    packets) alternating between two slabs with different strides, default
    gates and gate arrays -- every gate as the oracle's, nothing written
    past a ticket's packets"""
    n = 1 << 16
    keys, gates, frames = P.em_workload(1000, n, seed=21, pkt_seed=22)
    want_a = oracle_gates(keys, gates, frames, default_gate=8192)
    want_b = oracle_gates(keys, gates, frames, default_gate=77)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    f128 = np.zeros((n, 128), np.uint8)
    f128[:, :64] = frames.reshape(n, 64)
    da = torch.from_numpy(frames.reshape(-1)).cuda()
    db = torch.from_numpy(f128.reshape(-1)).cuda()
    ga = torch.full((n + 64,), -1, dtype=torch.int16, device="cuda")
    gb = torch.full((n + 64,), -1, dtype=torch.int16, device="cuda")
    rng = np.random.default_rng(23)
    ring = F.Ring(t, slots=1024)
    ca = cb = 0
    last = None
    while True:
        m = int(rng.integers(0, 301)) if rng.random() > 0.1 else 0
        if rng.random() < 0.5:
            m = min(m, n - ca)
            last = ring.submit(da, 64, m, 8192, ga, offset=ca)
            ca += m
        else:
            m = min(m, n - cb)
            last = ring.submit(db, 128, m, 77, gb, offset=cb)
            cb += m
        if ca == n and cb == n:
            break
    ring.wait(last)
    got_a = ga.cpu().numpy().view(np.uint16)
    got_b = gb.cpu().numpy().view(np.uint16)
    assert (got_a[:n] == want_a).all() and (got_b[:n] == want_b).all()
    assert (got_a[n:] == 0xFFFF).all() and (got_b[n:] == 0xFFFF).all()
    ring.close()


@pytest.mark.parametrize("n_rules", [300, 100000])
def test_wm_ring_vs_oracle(n_rules):
    """the ring over a WildcardMatch table (bg_wm_ring_create): its image
    probed in L2 (100 K rules: tag words, direct tuples) or held in LDS (300
    rules); batches of 32 / 100 / 4096 and per-ticket default gates, every
    gate as the oracle's WildcardMatch::ProcessBatch"""
    n = 1 << 16
    rk, rm, prio, wg, wf, _ = P.wm_workload(n_rules, n, stride=2048)
    frames = np.ascontiguousarray(wf[:, :64])
    fields = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]
    ow = O.OracleWildcardMatch(fields=fields)
    t = F.WmTable(P.FIVE_TUPLE)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, m, p, g in zip(rk, rm, prio, wg):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
        kb, mb = k.tobytes(), m.tobytes()
        ow.add(gate=int(g), priority=int(p), values=[{"value_bin": kb[a:c]} for a, c in cut],
               masks=[{"value_bin": mb[a:c]} for a, c in cut])
    want = ow.process(frames, 64, n)  # default gate: DROP_GATE (8192)
    hit = want != O.DROP_GATE
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    ring = F.Ring(t, slots=512)
    for burst in (32, 100, 4096):
        dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
        ring.run(d, 64, n, burst, 8192, dg)
        assert (dg.cpu().numpy().view(np.uint16) == want).all(), burst
    dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
    last = None
    for i, off in enumerate(range(0, n, 1000)):
        m = min(1000, n - off)
        last = ring.submit(d, 64, m, 77 if i % 2 else 8192, dg, offset=off)
    ring.wait(last)
    got = dg.cpu().numpy().view(np.uint16)
    dflt = np.where((np.arange(n) // 1000) % 2 == 1, 77, 8192)
    assert (got == np.where(hit, want, dflt)).all()
    ring.close()

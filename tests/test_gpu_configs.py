"""BASELINE configs at their own sizes through the HIP path, bit-exact
against the oracle; the drop-in module path under concurrent workers;
EmitPacket's per-gate batches and drops (core/module.h:534-618).

  C2: 1K-rule 5-tuple ExactMatch over the bench's 16,777,216 64 B packets;
  C3: IPChecksum -> L4Checksum over 1,048,576 1500 B frames in 2 KB slots,
      every byte of every frame compared;
  C5: 1,048,576-rule 5-tuple ExactMatch (table in HBM/MALL), as one image
      and as 8 partitions attached as one image (the multi-GPU build);
  C4: 100K-rule WildcardMatch over 8 masks on IMIX frames in 2 KB slots
      (tag words in LDS, and the key-filter path), and the bench's 8 M
      header-slab packets.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import _lib as LB  # noqa: E402
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).cuda()


def oracle_em_bulk(keys, gates):
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        assert L.or_em_add_field(em, off, size, 0, i, None, 0) == 0
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates, dtype=np.uint16)
    assert L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data) == 0
    return em


def oracle_em_gates(keys, gates, frames, stride, default_gate=8192):
    em = oracle_em_bulk(keys, gates)
    want = np.zeros(len(frames), np.uint16)
    O.lib().or_em_process(em, frames.ctypes.data, stride, len(frames),
                          default_gate, want.ctypes.data)
    O.lib().or_em_free(em)
    return want


@pytest.fixture(scope="module")
def c5():
    keys, gates, frames = P.em_workload(1 << 20, 1 << 21, seed=0xC5,
                                        pkt_seed=0xC55)
    want = oracle_em_gates(keys, gates, frames, 64)
    assert 0.4 < (want != 8192).mean() < 0.6
    return keys, gates, frames, want


# ------------------------------------------------------------------- C2
def test_c2_full_size():
    """the bench's C2 workload, all 16 M gates"""
    n = 16 << 20
    keys, gates, frames = P.em_workload(1000, n, seed=0x5EED)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d_g = torch.zeros(n, dtype=torch.int16, device="cuda")
    t.classify(to_dev(frames), 64, n, 8192, d_g)
    torch.cuda.synchronize()
    assert t.table_info()[1] == 1  # table in LDS
    want = oracle_em_gates(keys, gates, frames, 64)
    assert (d_g.cpu().numpy().view(np.uint16) == want).all()
    assert 0.4 < (want != 8192).mean() < 0.6


# ------------------------------------------------------------------- C3
def test_c3_full_size():
    """1 M 1500 B frames, IPChecksum -> L4Checksum recompute in one pass:
    both gate arrays and every frame byte"""
    n = 1 << 20
    cf = P.cksum_workload(n, frame_len=1496)
    d = to_dev(cf)
    ipg = torch.zeros(n, dtype=torch.int16, device="cuda")
    l4g = torch.zeros(n, dtype=torch.int16, device="cuda")
    F.cksum(d, 2048, n, 3, False, ipg, l4g)
    torch.cuda.synchronize()
    wip, wl4 = O.cksum_process(cf, 2048, n, 3, False)  # in place on the host copy
    assert (ipg.cpu().numpy().view(np.uint16) == wip).all()
    assert (l4g.cpu().numpy().view(np.uint16) == wl4).all()
    assert (d.cpu().numpy() == cf.reshape(-1)).all()


# ---------------------------------------------- ExactMatch on 1500 B packets
def test_em_1500b_full_size():
    """the north star's 1500 B match point (bench EM_1500B): C2's 1K rules
    over the bench's 4 M 1500 B packets (1496 B frames in 2 KB slots, the
    payload random here), every gate against the oracle run on the whole
    frames"""
    n = 1 << 22
    keys, gates, hdr = P.em_workload(1000, n, seed=0x5EED, stride=64,
                                     frame_len=1496, pkt_seed=0x1500)
    d = torch.randint(0, 256, (n, 2048), dtype=torch.uint8, device="cuda")
    d[:, :64] = torch.from_numpy(hdr).cuda()
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d_g = torch.zeros(n, dtype=torch.int16, device="cuda")
    t.classify(d.view(-1), 2048, n, 8192, d_g)
    got = d_g.cpu().numpy().view(np.uint16)
    # the oracle over whole 2 KB slots on a sample, over the header lines
    # (all it reads at these field offsets) for the rest
    k = 1 << 16
    full = d[:k].cpu().numpy()
    assert (full[:, :64] == hdr[:k]).all()
    assert (got[:k] == oracle_em_gates(keys, gates, full, 2048)).all()
    want = oracle_em_gates(keys, gates, hdr, 64)
    assert (got == want).all()
    assert 0.4 < (want != 8192).mean() < 0.6


# ------------------------------------------------------------------- C5
@pytest.mark.parametrize("flags", [0, LB.BG_PATH_NO_SLAB])
def test_c5_1m_rules_single_image(c5, flags):
    keys, gates, frames, want = c5
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    assert len(t) == 1 << 20
    d_g = torch.zeros(len(frames), dtype=torch.int16, device="cuda")
    with LB.kernel_paths(flags):
        t.classify(to_dev(frames), 64, len(frames), 8192, d_g)
        torch.cuda.synchronize()
    nbytes, in_lds = t.table_info()
    assert not in_lds and nbytes > 16 << 20
    assert (d_g.cpu().numpy().view(np.uint16) == want).all()


def test_c5_8_partitions_attached(c5):
    """the multi-GPU table: 8 partitions, each holding only its rules (as
    each rank inserts them), built separately and attached as one image"""
    keys, gates, frames, want = c5
    parts, counts = [], []
    for r in range(8):
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates, part=r, nparts=8)
        parts.append(t)
        counts.append(t.part_count(r, 8))
    assert sum(counts) == 1 << 20
    pb = [t.plan_count(8, max(counts)) for t in parts]
    assert len(set(pb)) == 1
    img = np.concatenate([t.build_part(r, pb[0]) for r, t in enumerate(parts)])
    full = F.EmTable(P.em_fields_5tuple())
    full.add_many(keys, gates)
    assert full.plan(8) == pb[0]
    d_img = to_dev(img)
    full.attach(0, d_img)
    d_g = torch.zeros(len(frames), dtype=torch.int16, device="cuda")
    full.classify(to_dev(frames), 64, len(frames), 8192, d_g)
    assert (d_g.cpu().numpy().view(np.uint16) == want).all()


# ------------------------------------------------------------------- C4
@pytest.mark.parametrize("flags", [0, LB.BG_PATH_WM_NO_JIT, LB.BG_PATH_WM_NO_TAGS])
def test_c4_imix_2k_slots(flags):
    """flags 0: the run-time compiled kernel (bg_wm_jit.cc) once ready;
    BG_PATH_WM_NO_JIT the ahead-of-time one; BG_PATH_WM_NO_TAGS the key
    filter"""
    n = 1 << 18
    rk, rm, prio, gates, frames, flen = P.wm_workload(100000, n, stride=2048)
    assert set(np.unique(flen)) == {60, 590, 1514}
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    assert t.num_tuples() == 8
    if flags == 0:
        t.jit_wait()
    d_g = torch.zeros(n, dtype=torch.int16, device="cuda")
    with LB.kernel_paths(flags):
        t.classify(to_dev(frames), 2048, n, 8192, d_g)
        torch.cuda.synchronize()
        in_lds = t.table_info()[1]
    assert in_lds == (2 if flags & LB.BG_PATH_WM_NO_TAGS else 3)  # key filter / tag words
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
        assert L.or_wm_add(ow, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    want = np.zeros(n, np.uint16)
    L.or_wm_process(ow, frames.ctypes.data, 2048, n, 8192, want.ctypes.data)
    L.or_wm_free(ow)
    assert (d_g.cpu().numpy().view(np.uint16) == want).all()
    assert (want != 8192).mean() > 0.3


def test_c4_header_slab_full_size():
    """the bench's C4 slab: 1 M IMIX frames' header lines, 8 copies (8 M
    packets), against the oracle on the frames themselves"""
    n0, rep = 1 << 20, 8
    rk, rm, prio, gates, frames, _ = P.wm_workload(100000, n0, stride=2048)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
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
        assert L.or_wm_add(ow, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    want = np.zeros(n0, np.uint16)
    L.or_wm_process(ow, frames.ctypes.data, 2048, n0, 8192, want.ctypes.data)
    L.or_wm_free(ow)
    h = to_dev(np.ascontiguousarray(frames[:, :64])).repeat(rep)
    del frames
    d_g = torch.zeros(n0 * rep, dtype=torch.int16, device="cuda")
    t.jit_wait()
    # run-time compiled, ahead-of-time
    for flags in (0, LB.BG_PATH_WM_NO_JIT):
        d_g.zero_()
        with LB.kernel_paths(flags):
            t.classify(h, 64, n0 * rep, 8192, d_g)
            torch.cuda.synchronize()
        # the /8 destination tuple is direct; the source port's 12.5 K rules
        # (a fifth of the 65536 ports) stay hashed (bg_api.cc kDirect2MinEntries)
        assert t.table_info()[1] == 3 and t.direct_tuples() == 1
        assert (d_g.cpu().numpy().view(np.uint16).reshape(rep, n0) == want).all(), flags


# ------------------------------------------- concurrent workers, one module
def _em_module_and_oracle(n_rules, n_pkts, seed):
    from bess_amd.modules import ExactMatch
    keys, gates, frames = P.em_workload(n_rules, n_pkts, seed=seed)
    fields = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]
    m = ExactMatch(fields=fields)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        m.add(fields=[{"value_bin": kb[a:c]} for a, c in cut], gate=int(g))
    want = oracle_em_gates(keys, gates, frames, 64)
    return m, frames, want


def test_concurrent_workers_one_module():
    """8 worker threads run the synchronous drop-in path (ProcessBatch of 32
    packets, bg_module_run) on ONE ExactMatch module at the same time, and 8
    more each drive their own bg_pipe over it; every gate equals the
    oracle's (core/module.h:485: lookups from many workers at once)."""
    from bess_amd.modules import Pipe
    m, frames, want = _em_module_and_oracle(1000, 1 << 16, seed=21)
    snb = np.zeros((len(frames), 2624), np.uint8)  # snbuf-like buffers
    snb[:, 512:512 + 64] = frames
    heads = snb.ctypes.data + 512 + 2624 * np.arange(len(frames), dtype=np.uintp)
    outs, errs = {}, []

    def sync_worker(w):
        try:
            rot = np.roll(np.arange(len(frames)), -w * 977)
            g = m.run(heads[rot], burst=32)
            outs[("sync", w)] = (rot, g)
        except Exception as e:  # reported below
            errs.append(e)

    def pipe_worker(w):
        try:
            rot = np.roll(np.arange(len(frames)), -w * 1231)
            p = Pipe(m, batch=2048, depth=3)
            g = p.run(heads[rot])
            p.close()
            outs[("pipe", w)] = (rot, g)
        except Exception as e:
            errs.append(e)

    ths = [threading.Thread(target=sync_worker, args=(w,)) for w in range(8)]
    ths += [threading.Thread(target=pipe_worker, args=(w,)) for w in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errs, errs
    assert len(outs) == 16
    for key, (rot, g) in outs.items():
        assert (g == want[rot]).all(), key


# ----------------------------------------------------- EmitPacket batches
def test_emit_batches_and_unconnected_gates():
    """Module::EmitPacket (core/module.h:543-594): packets join their
    gate's batch in order, a new batch starts at 32; a gate that is out of
    range (the default DROP_GATE 8192 on a miss) or not connected drops the
    packet (546-549)."""
    m, frames, want = _em_module_and_oracle(200, 3000, seed=23)
    n = len(frames)
    og, batches, dead = m.process_batches(frames, 64, n)
    w_og, w_b, w_dead = O.emit_packets(want)
    assert list(og) == w_og and batches == w_b and dead == w_dead
    assert dead and all(len(b) <= 32 for _, b in batches)
    conn = {0, 1, 2, 5}
    for g in conn:
        m.connect(g)
    og, batches, dead = m.process_batches(frames, 64, n)
    w_og, w_b, w_dead = O.emit_packets(want, connected=conn)
    assert list(og) == w_og and batches == w_b and dead == w_dead
    assert set(g for g, _ in batches) <= conn

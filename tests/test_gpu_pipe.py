"""Asynchronous host ingress/egress (bg_pipe_*): packets in snbuf-like host
buffers go through the aggregation queue in BESS-sized (<= 32) submits and
come back in submission order with the gate the reference's ProcessBatch
emits them to -- bit-exact against the oracle -- and, for the checksum
modules, with their recomputed checksum words written back in place."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import packets as P  # noqa: E402
from bess_amd.modules import (ExactMatch, IPChecksum, L4Checksum,  # noqa: E402
                              Pipe, WildcardMatch)
from oracle import oracle as O  # noqa: E402

SNBUF = 2624      # mempool object stride (core/snbuf_layout.h:34-68)
HEADROOM = 512    # frame at +512 in the object


def snbufs(frames, flen=None):
    """copy frames (n x stride) into snbuf-like objects; -> (buf, heads)"""
    n, w = frames.shape
    buf = np.zeros((n, SNBUF), np.uint8)
    m = min(w, SNBUF - HEADROOM)
    buf[:, HEADROOM:HEADROOM + m] = frames[:, :m]
    heads = buf.ctypes.data + HEADROOM + SNBUF * np.arange(n, dtype=np.uintp)
    return buf, heads


def run_pipe(pipe, heads, burst=32, lens=None, shuffle_seed=None):
    """ProcessBatch-style submits of `burst` packets, polling in between;
    cookies = packet index. Returns gates in packet order and checks the
    completion order is the submission order."""
    n = len(heads)
    order = np.arange(n, dtype=np.uintp)
    if shuffle_seed is not None:  # packets may arrive in any buffer order
        np.random.default_rng(shuffle_seed).shuffle(order)
    got_c, got_g = [], []
    for i in range(0, n, burst):
        idx = order[i:i + burst]
        pipe.submit(heads[idx], None if lens is None else lens[idx], idx)
        if (i // burst) % 7 == 0:
            c, g = pipe.poll(wait=False)
            got_c.append(c)
            got_g.append(g)
    c, g = pipe.drain()
    got_c.append(c)
    got_g.append(g)
    c = np.concatenate(got_c)
    g = np.concatenate(got_g)
    assert (c == order).all(), "completion order != submission order"
    out = np.empty(n, np.uint16)
    out[c.astype(np.int64)] = g
    return out


FIELDS = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]


def em_pair(keys, gates):
    m = ExactMatch(fields=FIELDS)
    om = O.OracleExactMatch(fields=FIELDS)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        vals = [{"value_bin": kb[a:c]} for a, c in cut]
        m.add(fields=vals, gate=int(g))
        om.add(fields=vals, gate=int(g))
    m.set_default_gate(gate=64)
    om.set_default_gate(64)
    return m, om


@pytest.mark.parametrize("mode", ["ring", "launch"])
@pytest.mark.parametrize("batch,depth,burst", [(4096, 4, 32), (1000, 2, 32),
                                               (1, 1, 3), (65536, 3, 32),
                                               (1024, 8, 32)])
def test_em_pipe_vs_oracle(batch, depth, burst, mode):
    """ring: the slots go to the module's persistent kernel (the default
    for ExactMatch); launch: H2D / kernel / D2H per slot"""
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        _em_pipe_vs_oracle(batch, depth, burst)


def _em_pipe_vs_oracle(batch, depth, burst):
    n = 20000 if batch > 1 else 500
    keys, gates, frames = P.em_workload(1000, n, seed=11)
    m, om = em_pair(keys, gates)
    want = om.process(frames, 64, n)
    buf, heads = snbufs(frames)
    pipe = Pipe(m, batch=batch, depth=depth)
    lo, hi, st = pipe.window()
    assert (lo, hi, st) == (23, 38, 16)  # only the field window travels
    got = run_pipe(pipe, heads, burst=burst, shuffle_seed=batch)
    assert (got == want).all()
    # a rule change between batches is seen by the next launch
    m.set_default_gate(gate=5)
    om.set_default_gate(5)
    k = min(n, 3000)
    got = run_pipe(pipe, heads[:k], burst=burst)
    assert (got == om.process(frames[:k], 64, k)).all()
    pipe.close()


@pytest.mark.parametrize("mode", ["ring", "launch"])
def test_module_destroyed_before_its_pipe(mode):
    """bg_module_destroy with a pipe still open (a host tearing its graph
    down in any order, or Python's collector freeing a cycle): the module
    stays alive until the pipe goes, and the pipe keeps classifying"""
    import ctypes as C
    from bess_amd._lib import kernel_paths, lib, BG_PATH_PIPE_NO_RING
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        n = 5000
        keys, gates, frames = P.em_workload(200, n, seed=13)
        m, om = em_pair(keys, gates)
        want = om.process(frames, 64, n)
        buf, heads = snbufs(frames)
        pipe = Pipe(m, batch=1024, depth=2)
        got1 = run_pipe(pipe, heads[:2000])
        lib().bg_module_destroy(m.h)  # the owner lets go first
        m.h = None
        got2 = run_pipe(pipe, heads[2000:])
        pipe.close()
        assert (np.concatenate([got1, got2]) == want).all()


def test_ring_pipe_refilled_slots():
    """ring mode with slots refilled many times: each refill's windows must
    be read fresh by the persistent kernel (no line of an earlier batch
    served from the device's caches), over several rounds of the same slots"""
    n = 60000
    keys, gates, frames = P.em_workload(1000, n, seed=14)
    m, om = em_pair(keys, gates)
    want = om.process(frames, 64, n)
    buf, heads = snbufs(frames)
    pipe = Pipe(m, batch=512, depth=2)
    for rnd in range(3):
        got = run_pipe(pipe, heads, shuffle_seed=100 + rnd)
        assert (got == want).all(), rnd
    pipe.close()


@pytest.mark.parametrize("mode", ["ring", "launch"])
@pytest.mark.parametrize("cls", ["em", "wm"])
def test_pipe_metadata_fields_vs_oracle(mode, cls):
    """attr_name fields on the aggregation queue: each packet's metadata
    bytes travel in its staged row after the field window (frames and
    metadata areas in separate host buffers), bit-exact against the oracle;
    submitting without metadata is refused"""
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    from bess_amd.modules import ModuleError
    from test_attr_fields import (ATTR_OFF, EM_FIELDS, EM_MASKS, META_OFF, STRIDE,
                                  em_rules, slots)
    n = 30000
    f = slots(n, 61)
    if cls == "em":
        o = O.OracleExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
        m = ExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
        for vals, g in em_rules(o, f, 2000, np.random.default_rng(62)):
            o.add(fields=vals, gate=g)
            m.add(fields=vals, gate=g)
    else:
        fields = [{"attr_name": "foo", "num_bytes": 2}, {"offset": 30, "num_bytes": 4},
                  {"attr_name": "bar", "num_bytes": 1}]
        o = O.OracleWildcardMatch(fields=fields)
        m = WildcardMatch(fields=fields)
        rng = np.random.default_rng(63)
        for i in rng.choice(n, 500, replace=False):
            src = [f[i, META_OFF + 8:META_OFF + 10].tobytes(), f[i, 30:34].tobytes(),
                   f[i, META_OFF + 21:META_OFF + 22].tobytes()]
            mk = [b"\xff\xff", b"\xff\xff\x00\x00", b"\x03"]
            arg = dict(gate=int(rng.integers(0, 64)), priority=int(rng.integers(0, 5)),
                       values=[{"value_bin": bytes(x & y for x, y in zip(s_, mb))}
                               for s_, mb in zip(src, mk)],
                       masks=[{"value_bin": mb} for mb in mk])
            o.add(**arg)
            m.add(**arg)
    want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=ATTR_OFF)
    frames = np.ascontiguousarray(f[:, :META_OFF])
    meta = np.ascontiguousarray(f[:, META_OFF:])
    heads = frames.ctypes.data + META_OFF * np.arange(n, dtype=np.uintp)
    metas = meta.ctypes.data + (STRIDE - META_OFF) * np.arange(n, dtype=np.uintp)
    m.bind_meta(-1, ATTR_OFF)
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        pipe = Pipe(m, batch=1024, depth=4)
        with pytest.raises(ModuleError):
            pipe.submit(heads[:8])
        order = np.random.default_rng(64).permutation(n).astype(np.uintp)
        cs, gs = [], []
        for i in range(0, n, 32):
            idx = order[i:i + 32]
            pipe.submit(heads[idx], cookies=idx, metas=metas[idx])
            c, g = pipe.poll()
            cs.append(c)
            gs.append(g)
        c, g = pipe.drain()
        pipe.close()
    c = np.concatenate(cs + [c])
    g = np.concatenate(gs + [g])
    assert (c == order).all()
    got = np.empty(n, np.uint16)
    got[c.astype(np.int64)] = g
    assert (got == want).all() and (want != O.DROP_GATE).mean() > 0.02


@pytest.mark.parametrize("mode", ["ring", "launch"])
@pytest.mark.parametrize("cls", ["em", "wm"])
def test_pipe_rebind_permuted_attr_offsets(mode, cls):
    """A pipeline change that swaps two attributes' metadata offsets but
    keeps their window [mlo, mhi): pipes opened after the re-bind read each
    attribute at its new offset (a ring built for the old layout must not be
    reused), bit-exact against the oracle under each layout"""
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    from test_attr_fields import META_OFF, STRIDE, slots
    fields = [{"attr_name": "foo", "num_bytes": 4}, {"attr_name": "bar", "num_bytes": 4},
              {"offset": 26, "num_bytes": 2}]
    lay1, lay2 = {"foo": 8, "bar": 12}, {"foo": 12, "bar": 8}
    n = 20000
    f = slots(n, 71)
    rng = np.random.default_rng(72)
    if cls == "em":
        o, m = O.OracleExactMatch(fields=fields), ExactMatch(fields=fields)
    else:
        o, m = O.OracleWildcardMatch(fields=fields), WildcardMatch(fields=fields)
    for i in rng.choice(n, 1500, replace=False):
        lay = lay1 if i % 2 else lay2  # rules that match under either layout
        vals = [{"value_bin": f[i, META_OFF + lay["foo"]:META_OFF + lay["foo"] + 4].tobytes()},
                {"value_bin": f[i, META_OFF + lay["bar"]:META_OFF + lay["bar"] + 4].tobytes()},
                {"value_bin": f[i, 26:28].tobytes()}]
        g = int(rng.integers(0, 64))
        if cls == "em":
            o.add(fields=vals, gate=g)
            m.add(fields=vals, gate=g)
        else:
            mk = [{"value_bin": b"\xff" * 4}, {"value_bin": b"\xff" * 4},
                  {"value_bin": b"\xff\xff"}]
            o.add(values=vals, masks=mk, gate=g, priority=1)
            m.add(values=vals, masks=mk, gate=g, priority=1)
    frames = np.ascontiguousarray(f[:, :META_OFF])
    meta = np.ascontiguousarray(f[:, META_OFF:])
    heads = frames.ctypes.data + META_OFF * np.arange(n, dtype=np.uintp)
    metas = meta.ctypes.data + (STRIDE - META_OFF) * np.arange(n, dtype=np.uintp)
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        for lay in (lay1, lay2, lay1):
            want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=lay)
            m.bind_meta(-1, lay)
            pipe = Pipe(m, batch=1024, depth=3)
            cs, gs = [], []
            for i in range(0, n, 32):
                idx = np.arange(i, min(n, i + 32), dtype=np.uintp)
                pipe.submit(heads[idx], cookies=idx, metas=metas[idx])
                c, g = pipe.poll()
                cs.append(c)
                gs.append(g)
            c, g = pipe.drain()
            pipe.close()
            got = np.empty(n, np.uint16)
            got[np.concatenate(cs + [c]).astype(np.int64)] = np.concatenate(gs + [g])
            assert (got == want).all(), lay
            assert (want != O.DROP_GATE).mean() > 0.03


def test_em_pipes_share_ring_lanes():
    """18 pipes on one module, each run by its own thread (as bessd workers
    submit): more pipes than the module's ring has lanes (16), so two pairs
    share a lane; every packet's gate is bit-exact"""
    import threading
    n = 16384
    keys, gates, frames = P.em_workload(1000, n, seed=12)
    m, om = em_pair(keys, gates)
    want = om.process(frames, 64, n)
    buf, heads = snbufs(frames)
    pipes = [Pipe(m, batch=1024, depth=8) for _ in range(18)]
    outs, errs = [None] * len(pipes), []

    def work(i):
        try:
            outs[i] = pipes[i].run(heads)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(pipes))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for p in pipes:
        p.close()
    assert not errs, errs
    for o in outs:
        assert (o == want).all()


@pytest.mark.parametrize("mode", ["ring", "launch"])
@pytest.mark.parametrize("n_rules,batch,depth", [(2000, 2048, 3), (100000, 1024, 8),
                                                 (300, 512, 2)])
def test_wm_pipe_vs_oracle(n_rules, batch, depth, mode):
    """ring: the slots go to the module's persistent WildcardMatch kernel
    (its own image copy probed in L2, or in LDS for a small table: 300
    rules); launch: H2D / kernel / D2H per slot. A rule change and a new
    default gate between batches are seen by the next slots (a new ring)"""
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    rk, rm, prio, wg, wf, flen = P.wm_workload(n_rules, 12000, stride=2048)
    m = WildcardMatch(fields=FIELDS)
    ow = O.OracleWildcardMatch(fields=FIELDS)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]

    def add(k, mk, p, g):
        kb, mb = k.tobytes(), mk.tobytes()
        kw = dict(gate=int(g), priority=int(p),
                  values=[{"value_bin": kb[a:c]} for a, c in cut],
                  masks=[{"value_bin": mb[a:c]} for a, c in cut])
        m.add(**kw)
        ow.add(**kw)
    half = len(rk) // 2
    for r in zip(rk[:half], rm[:half], prio[:half], wg[:half]):
        add(*r)
    _, heads = snbufs(wf)
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        pipe = Pipe(m, batch=batch, depth=depth)
        got = run_pipe(pipe, heads, shuffle_seed=n_rules)
        assert (got == ow.process(wf, 2048, len(wf))).all()
        for r in zip(rk[half:], rm[half:], prio[half:], wg[half:]):
            add(*r)
        m.set_default_gate(gate=7)
        ow.set_default_gate(7)
        got = run_pipe(pipe, heads)
        want = ow.process(wf, 2048, len(wf))
        assert (got == want).all() and (want == 7).any()
        pipe.close()


@pytest.mark.parametrize("cls,mode", [(IPChecksum, 1), (L4Checksum, 2)])
@pytest.mark.parametrize("verify", [False, True])
def test_cksum_pipe_writeback_vs_oracle(cls, mode, verify):
    n = 6000
    frames = P.cksum_workload(n, frame_len=590)
    if verify:  # half the frames carry correct checksums
        O.cksum_process(frames[:n // 2], 2048, n // 2, 3, False)
    ref = frames.copy()
    ipg, l4g = O.cksum_process(ref, 2048, n, mode, verify)
    want = ipg if mode == 1 else l4g
    buf, heads = snbufs(frames)
    lens = np.full(n, 590, np.uint16)
    pipe = Pipe(cls(verify=verify), batch=1024, depth=3, span=1504)
    got = run_pipe(pipe, heads, lens=lens, shuffle_seed=1)
    assert (got == want).all()
    # the recomputed header line went back into every packet buffer, and
    # nothing else in the buffer changed
    out = buf[:, 512:512 + 2048]
    assert (out[:, :590] == ref[:, :590]).all()
    assert (buf[:, :512] == 0).all() and (out[:, 590:] == frames[:, 590:]).all()


@pytest.mark.parametrize("cls,mode", [(IPChecksum, 1), (L4Checksum, 2)])
@pytest.mark.parametrize("verify", [False, True])
def test_cksum_pipe_p11_bytes_past_data_len(cls, mode, verify):
    """A frame's length fields past its data_len: the pipe stages the bytes
    the reference reads (Module::StageReach), so the checksum words and
    gates equal the oracle's over the whole buffers -- round 4's pipe
    zero-padded past data_len and summed zeros there."""
    n = 3000
    frames, lens = P.cksum_p11_workload(n)
    if verify:  # half the frames carry the checksums of their full buffers
        O.cksum_process(frames[:n // 2], 2048, n // 2, 3, False)
    ref = frames.copy()
    ipg, l4g = O.cksum_process(ref, 2048, n, mode, verify)
    want = ipg if mode == 1 else l4g
    buf, heads = snbufs(frames)
    pipe = Pipe(cls(verify=verify), batch=512, depth=3)
    got = run_pipe(pipe, heads, lens=lens, shuffle_seed=3)
    pipe.close()
    assert (got == want).all()
    if verify:
        assert (want == 0).any() and (want == 1).any()
    out = buf[:, 512:512 + 2048]
    assert (out == ref).all()


@pytest.mark.parametrize("cls,mode", [(IPChecksum, 1), (L4Checksum, 2)])
@pytest.mark.parametrize("verify", [False, True])
def test_cksum_pipe_zero_copy_vs_oracle(cls, mode, verify):
    """Packets in host-registered memory (bg_host_register: the packet
    pool): the pipe hands the device their head pointers and the kernel
    works on the buffers in place -- including the bytes past data_len the
    reference reads (P11) -- with unregistered packets (copied, zero-padded
    past what they read) interleaved, so slots switch kind; every gate and
    every byte of the data areas as the oracle gives them."""
    from bess_amd.flowtable import HostRegion
    n = 3000
    frames, lens = P.cksum_p11_workload(n, seed=17)
    if verify:
        O.cksum_process(frames[:n // 2], 2048, n // 2, 3, False)
    ref = frames.copy()
    ipg, l4g = O.cksum_process(ref, 2048, n, mode, verify)
    want = ipg if mode == 1 else l4g
    buf, heads = snbufs(frames)
    reg = HostRegion(buf)
    try:
        # a third of the packets from a copy that is not registered
        other = np.random.default_rng(3).random(n) < 1 / 3
        buf2, heads2 = snbufs(frames)
        heads = np.where(other, heads2, heads)
        pipe = Pipe(cls(verify=verify), batch=512, depth=3)
        got = run_pipe(pipe, heads, lens=lens, shuffle_seed=5)
        pipe.close()
    finally:
        reg.close()
    assert (got == want).all()
    out = np.where(other[:, None], buf2, buf)[:, 512:512 + 2048]
    assert (out == ref).all()


@pytest.mark.parametrize("cls,mode", [(IPChecksum, 1), (L4Checksum, 2)])
def test_cksum_pipe_zero_copy_unaligned_heads(cls, mode):
    """Registered packets whose heads are not 16-byte aligned (data_off moved
    by prepend / adj: +2, +4, +8) beside aligned ones: the aligned go in
    place, the others are staged (the kernel's frame loads are 16-byte);
    every gate and every byte as the oracle gives them"""
    from bess_amd.flowtable import HostRegion
    n = 3000
    frames, lens = P.cksum_p11_workload(n, seed=29)
    ref = frames.copy()
    ipg, l4g = O.cksum_process(ref, 2048, n, mode, False)
    want = ipg if mode == 1 else l4g
    off = np.random.default_rng(4).choice([0, 2, 4, 8], n)
    buf = np.zeros((n, SNBUF), np.uint8)
    for i in range(n):
        buf[i, HEADROOM + off[i]:HEADROOM + off[i] + 2048] = frames[i]
    heads = (buf.ctypes.data + HEADROOM + off + SNBUF * np.arange(n)).astype(np.uintp)
    reg = HostRegion(buf)
    try:
        pipe = Pipe(cls(verify=False), batch=512, depth=3)
        got = run_pipe(pipe, heads, lens=lens, shuffle_seed=6)
        pipe.close()
    finally:
        reg.close()
    assert (got == want).all()
    for i in range(n):
        assert (buf[i, HEADROOM + off[i]:HEADROOM + off[i] + 2048] == ref[i]).all(), i


def test_cksum_ptrs_device_and_host_memory():
    """bg_cksum_ptrs over frames by pointer: device memory in a permuted
    order, and host-registered memory, against the oracle"""
    from bess_amd import flowtable as F
    from bess_amd.flowtable import HostRegion
    n = 5000
    frames, _ = P.cksum_p11_workload(n, seed=23)
    ref = frames.copy()
    ipg, l4g = O.cksum_process(ref, 2048, n, 3, False)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    perm = np.random.default_rng(1).permutation(n)
    ptrs = torch.from_numpy((d.data_ptr() + 2048 * perm).astype(np.uint64).view(np.int64)).cuda()
    gi = torch.zeros(n, dtype=torch.int16, device="cuda")
    gl = torch.zeros(n, dtype=torch.int16, device="cuda")
    F.cksum_ptrs(ptrs, 2048, n, 3, False, gi, gl)
    torch.cuda.synchronize()
    assert (gi.cpu().numpy().view(np.uint16) == ipg[perm]).all()
    assert (gl.cpu().numpy().view(np.uint16) == l4g[perm]).all()
    assert (d.cpu().numpy().reshape(n, 2048) == ref).all()
    h = frames.copy()
    reg = HostRegion(h)
    try:
        hp = np.array([reg.addr(h.ctypes.data + 2048 * i, 2048) for i in perm], np.uint64)
        F.cksum_ptrs(torch.from_numpy(hp.view(np.int64)).cuda(), 2048, n, 3, False, gi, gl)
        torch.cuda.synchronize()
    finally:
        reg.close()
    assert (gl.cpu().numpy().view(np.uint16) == l4g[perm]).all()
    assert (h == ref).all()


def test_pipe_empty_and_flush():
    keys, gates, frames = P.em_workload(10, 10, seed=2)
    m, om = em_pair(keys, gates)
    pipe = Pipe(m, batch=64, depth=2)
    pipe.flush()
    c, g = pipe.poll(wait=True)
    assert len(c) == 0 and pipe.pending() == 0
    _, heads = snbufs(frames)
    pipe.submit(heads[:5])
    assert pipe.pending() == 5
    c, g = pipe.poll(wait=True)  # nothing launched yet: the slot is partial
    assert len(c) == 0
    c, g = pipe.drain()
    assert (g == om.process(frames[:5], 64, 5)).all()
    assert (c == heads[:5]).all()  # default cookie: the head pointer
